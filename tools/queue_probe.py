"""How HIP streams map onto hardware queues (GPU_MAX_HW_QUEUES): N streams,
normal or high priority, each given one long torch.cuda._sleep kernel at
once; the wall time shows how many ran concurrently (development tool;
run under rocprofv3 --kernel-trace to see Queue_Id per stream)."""
import sys
import time

import torch


def run(n, prio):
    ss = [torch.cuda.Stream(priority=prio) for _ in range(n)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in ss:
        with torch.cuda.stream(s):
            torch.cuda._sleep(50_000_000)
    torch.cuda.synchronize()
    return time.perf_counter() - t0


torch.cuda.init()
one = run(1, 0)
print("one sleep kernel: %.1f ms" % (one * 1e3))
for prio in (0, -1):
    for n in (2, 3, 4, 6, 8):
        dt = run(n, prio)
        print("prio %2d  %d streams: %.1f ms = %.2f x one" % (prio, n, dt * 1e3, dt / one), flush=True)
