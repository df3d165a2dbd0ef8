#!/usr/bin/env python3
"""PCIe duplex probe: host->device and device->host copy rates of pinned
buffers, each alone and both at once on two streams (what the host-to-host
leg needs: chunk k + 1's upload under chunk k's download).

    python tools/duplex_probe.py [MiB]
"""
import json
import sys
import time

import torch


def main():
    mib = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    n = mib << 20
    dev = torch.device("cuda", 0)
    h_up = torch.empty(n, dtype=torch.uint8).pin_memory()
    h_dn = torch.empty(n, dtype=torch.uint8).pin_memory()
    d_up = torch.empty(n, dtype=torch.uint8, device=dev)
    d_dn = torch.empty(n, dtype=torch.uint8, device=dev)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    out = {"bytes": n}

    def timed(fn, reps=5):
        best = 1e9
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t0)
        return best

    def up():
        with torch.cuda.stream(s1):
            d_up.copy_(h_up, non_blocking=True)

    def dn():
        with torch.cuda.stream(s2):
            h_dn.copy_(d_dn, non_blocking=True)

    def both():
        up()
        dn()

    t = timed(up)
    out["h2d_GBps"] = round(n / t / 1e9, 1)
    t = timed(dn)
    out["d2h_GBps"] = round(n / t / 1e9, 1)
    t = timed(both)
    out["both_ms"] = round(t * 1e3, 2)
    out["both_aggregate_GBps"] = round(2 * n / t / 1e9, 1)
    out["duplex_factor"] = round((n / out["h2d_GBps"] + n / out["d2h_GBps"]) / 1e9 / t, 2)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
