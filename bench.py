#!/usr/bin/env python3
"""bench.py — FLAC-8 batch encode throughput on MI355X (BASELINE.json config 2).

One step = one pass of the hot path over one batch: FLAC-8 encode of
`--tracks` synthetic 44.1 kHz / 16-bit stereo tracks x `--frames` FLAC
frames of 4096 PCM frames, PCM resident in HBM, complete .flac images
(STREAMINFO with MD5, VORBIS_COMMENT, PADDING, frames) left in HBM.

Multi-GPU: one process per GPU (torchrun); each rank encodes its own batch
of `--tracks` tracks (tracks are independent, no collective on the data
path) -> "scaling": "weak"; value = frames of all ranks / max-over-ranks time.

Prints ONE JSON line on rank 0.  The roofline block is for the dominant
kernel (timed with HIP events on the stream it runs on, inside libatgpu);
cpu_baseline times the CPU oracle (oracle/flac_port.c) on a bounded sample
of the same batch on this host's cores.
"""
import argparse
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "python-audio-tools_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

METRIC = "FLAC-8 encode frames/s (4096-sample 44.1k stereo) at 1/2/4/8 GPUs; bit-exact"
BLOCK = 4096
PCM_BYTES_PER_FRAME = BLOCK * 2 * 2
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
FLAC8 = dict(block_size=4096, max_lpc_order=12, min_residual_partition_order=0,
             max_residual_partition_order=6, mid_side=True,
             exhaustive_model_search=True)


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--tracks", type=int, default=1024)
    ap.add_argument("--frames", type=int, default=64, help="FLAC frames per track")
    ap.add_argument("--cpu-sample-tracks", type=int, default=1024)
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--no-decode", action="store_true",
                    help="skip the decode leg (GPU FLAC decode of the encoded batch)")
    return ap.parse_args(argv)


def shard(n_total_ranks, rank, tracks_per_rank):
    """global track ids owned by `rank` (weak scaling: a full batch per rank;
    tracks are independent, so ranks share nothing on the data path)"""
    return list(range(rank * tracks_per_rank, (rank + 1) * tracks_per_rank))


def reduce_max(torch, dist, value, device):
    """max of a host float over all ranks (the step clock: max over ranks)"""
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def synth_batch(torch, track_ids, n_samples, device):
    """seeded synthetic PCM, int16 interleaved stereo, generated on device.

    SURVEY §8(d): per track two sines (f1 in [100,2000] Hz, f2 in [2k,12k] Hz,
    a1 + a2 <= 0.9) + gaussian noise sigma 64 LSB, right channel with
    frequencies x1.3; 5% white-noise tracks, 2% silent tracks."""
    T = len(track_ids)
    rs = [np.random.RandomState(0x5EED0000 + t) for t in track_ids]
    f1 = torch.tensor([r.uniform(100, 2000) for r in rs], dtype=torch.float64, device=device)
    f2 = torch.tensor([r.uniform(2000, 12000) for r in rs], dtype=torch.float64, device=device)
    a1 = torch.tensor([r.uniform(0.05, 0.6) for r in rs], dtype=torch.float64, device=device)
    a2 = torch.tensor([r.uniform(0.0, 0.3) for r in rs], dtype=torch.float64, device=device)
    kind = torch.tensor([(t * 2654435761) % 100 for t in track_ids], device=device)
    gen = torch.Generator(device=device)
    gen.manual_seed(0x5EED + track_ids[0])
    out = torch.empty((T, n_samples, 2), dtype=torch.int16, device=device)
    chunk = 64
    n = torch.arange(n_samples, dtype=torch.float64, device=device)
    for c0 in range(0, T, chunk):
        sl = slice(c0, min(T, c0 + chunk))
        ph = 2 * np.pi * n[None, :] / 44100.0
        for ch, fm in ((0, 1.0), (1, 1.3)):
            x = (a1[sl, None] * torch.sin(ph * f1[sl, None] * fm) +
                 a2[sl, None] * torch.sin(ph * f2[sl, None] * fm)) * 32767.0
            x = x + torch.randn(x.shape, generator=gen, device=device,
                                dtype=torch.float64) * 64.0
            x = torch.round(x).clamp_(-32768, 32767)
            wn = kind[sl] < 5
            if bool(wn.any()):
                u = torch.randint(-32768, 32768, x.shape, generator=gen, device=device)
                x = torch.where(wn[:, None], u.to(x.dtype), x)
            sil = (kind[sl] >= 5) & (kind[sl] < 7)
            x = torch.where(sil[:, None], torch.zeros_like(x), x)
            out[sl, :, ch] = x.to(torch.int16)
    return out.reshape(-1)


def cpu_baseline(pcm_host, n_tracks, samples_per_track, threads):
    """oracle FLAC-8 encode of `n_tracks` tracks on `threads` host threads
    (one track per thread at a time, like track2track -j N)"""
    import oracle_port
    oracle_port.load()
    work = list(range(n_tracks))
    lock = threading.Lock()

    def run():
        while True:
            with lock:
                if not work:
                    return
                t = work.pop()
            p = pcm_host[t * samples_per_track * 2:(t + 1) * samples_per_track * 2]
            oracle_port.encode(p.astype(np.int32), 2, 16, 44100, **FLAC8)

    th = [threading.Thread(target=run) for _ in range(threads)]
    t0 = time.perf_counter()
    for x in th:
        x.start()
    for x in th:
        x.join()
    dt = time.perf_counter() - t0
    frames = n_tracks * (samples_per_track // BLOCK)
    return frames / dt, dt


def cpu_decode_baseline(images, threads):
    """oracle FLAC decode (oracle/flac_port.c, pinned to the reference
    decoder) of `images` on `threads` host threads, one image per thread"""
    import oracle_port
    work = list(range(len(images)))
    lock = threading.Lock()
    nfr = [0]

    def run():
        while True:
            with lock:
                if not work:
                    return
                t = work.pop()
            r = oracle_port.decode_frames(images[t])
            with lock:
                nfr[0] += len(r["offsets"])

    th = [threading.Thread(target=run) for _ in range(threads)]
    t0 = time.perf_counter()
    for x in th:
        x.start()
    for x in th:
        x.join()
    dt = time.perf_counter() - t0
    return nfr[0] / dt, dt


def decode_leg(args, torch, dist, world, device, out, res, header, n_frames, barrier):
    """GPU decode of the batch the encoder just left in HBM (the trackverify
    path): every track is decoded, its PCM restored and
    its STREAMINFO MD5 checked on the GPU.  Returns the JSON object."""
    from audiotools import _atgpu
    dec = _atgpu.Decoder(int(os.environ.get("LOCAL_RANK", "0")))
    tracks = []
    for r in res:
        si = _atgpu.StreamInfo()
        si.total_samples = args.frames * BLOCK
        si.sample_rate, si.channels, si.bits_per_sample = 44100, 2, 16
        si.max_block_size = BLOCK
        si.md5[:] = bytes(r.md5)
        tracks.append(_atgpu.dec_track(r.out_offset + header, r.bytes - header, si))
    nbytes = max(r.out_offset + r.bytes for r in res)

    def step():
        return dec.decode_device(out.data_ptr(), nbytes, tracks)

    for _ in range(args.warmup):
        dres, _, _ = step()
    kt_sum = {}
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        dres, d_pcm, nsamp = step()
        for k, v in dec.kernel_times().items():
            kt_sum[k] = kt_sum.get(k, 0.0) + v
    barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        elapsed = reduce_max(torch, dist, elapsed, device)
    kt = {k: v / args.steps for k, v in kt_sum.items()}
    ok = all(r.status == 0 and r.pcm_frames == args.frames * BLOCK for r in dres)
    comp = sum(int(r.bytes) - header for r in res)
    pcm32 = args.tracks * args.frames * BLOCK * 2 * 4
    # algorithmic bytes per launch: the parsers read the compressed frames
    # once; the subframe decoder also writes its int32 row scratch, which
    # the row transposer reads and writes as planar samples; the
    # interleaver reads those and writes int32 PCM + the s16 byte stream
    alg = {"dec_scan": comp, "dec_parse": comp, "dec_chain": 0,
           "dec_subframe": comp + pcm32, "dec_unrow": 2 * pcm32,
           "dec_interleave": pcm32 * 2 + pcm32 // 2, "dec_md5": pcm32 // 2}
    kernels = {k: v for k, v in kt.items() if k in alg}
    dom = max(kernels, key=kernels.get)
    achieved = alg[dom] / (kernels[dom] / 1e3) / 1e9
    traffic = None
    tf = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(tf):
        try:
            traffic = json.load(open(tf)).get(dom)
        except Exception:
            traffic = None
    dec.close()
    return {
        "metric": "FLAC-8 decode frames/s (GPU decode of the encoded batch, MD5-verified)",
        "value": round(n_frames * world * args.steps / elapsed, 1), "unit": "frames/s",
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "kernel_ms": {k: round(v, 4) for k, v in kt.items()},
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 2),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                     "alg_bytes_per_launch": alg[dom], "launch_ms": round(kernels[dom], 4)},
        "verified_md5_round_trip": ok,
    }


def convert_leg(args, torch, device, pcm):
    """BPSConverter 16 -> 8 bits with dither over the whole batch
    (pcm_convert.hip): an HBM stream -- 4 B in + 4 B out +
    1/8 B of dither per sample.  Timed with torch's default-stream sync
    around the launches (the converter runs on the default stream)."""
    from audiotools import _atgpu
    lib = _atgpu.load_library()
    x = pcm.to(torch.int32)
    y = torch.empty_like(x)
    dither = torch.randint(0, 256, ((x.numel() + 7) // 8,), dtype=torch.uint8,
                           device=device)
    frames = x.numel() // 2

    def run():
        st = lib.atg_pcm_convert_device(_atgpu.CONV_BPS, x.data_ptr(), y.data_ptr(), frames,
                                        2, 0, 16, 8, dither.data_ptr(), 0, None)
        if st != _atgpu.ATG_OK:
            raise RuntimeError(lib.atg_pcm_convert_last_error())

    for _ in range(args.warmup):
        run()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        run()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.steps
    ok = bool((((y ^ (x >> 8)) & ~1) == 0).all().item())
    alg = x.numel() * 8 + dither.numel()
    del x, y, dither
    return {"metric": "BPSConverter 16->8 dither, samples/s", "value": round(frames * 2 / dt, 1),
            "unit": "samples/s", "ms_per_step": round(dt * 1e3, 4),
            "roofline": {"bound": "hbm", "kernel": "k_pcm_bps",
                         "achieved": round(alg / dt / 1e9, 2), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(alg / dt / 1e9 / HBM_PEAK_GBS, 4),
                         "traffic": None, "alg_bytes_per_launch": alg,
                         "launch_ms": round(dt * 1e3, 4)},
            "verified_dither_invariant": ok}


def album_reduce(dist, world, hist, peak):
    """an album spread over ranks: SUM of the uint32 window histograms (held
    as int32; two's-complement sums are the same bits) and MAX of the peak,
    in place -- exact and order-independent (SURVEY 8(e) ReplayGain row)"""
    if world > 1:
        dist.all_reduce(hist, op=dist.ReduceOp.SUM)
        dist.all_reduce(peak, op=dist.ReduceOp.MAX)


def replaygain_leg(args, torch, dist, world, rank, device, pcm, barrier):
    """ReplayGain title analysis of every track of the batch (replaygain.hip,
    SURVEY 8(a) G1-G5) plus one album over ALL ranks' tracks: each rank sums
    its tracks' window histograms on the GPU, then the 12000-bin uint32
    histogram is all-reduced (SUM, exact) and the album peak (MAX) over RCCL
    -- the one real exchange step of the path.  Returns the
    JSON object (rank 0) and per-track results for the CPU check."""
    from audiotools import _atgpu
    x = pcm.to(torch.int32)
    n_samples = args.frames * BLOCK
    tracks = [_atgpu.RgTrack(t * n_samples, n_samples, 2, 16, 44100, 0)
              for t in range(args.tracks)]
    hist = torch.zeros(12000, dtype=torch.int32, device=device)

    def step():
        res, peaks = _atgpu.replaygain_device(x.data_ptr(), tracks, 1, hist.data_ptr())
        pk = torch.tensor([peaks[0]], dtype=torch.float64, device=device)
        album_reduce(dist, world, hist, pk)
        gain = _atgpu.replaygain_hist_gain(hist.data_ptr(), 1)[0]
        return res, gain, float(pk.item())

    for _ in range(args.warmup):
        step()
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res, album_gain, album_peak = step()
    barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        elapsed = reduce_max(torch, dist, elapsed, device)
    host = pcm[:4 * n_samples * 2].cpu().numpy().astype(np.int32)
    del x
    frames = args.tracks * args.frames * world * args.steps
    out = {"metric": "ReplayGain title analysis, FLAC-frame-equivalents/s (4096 PCM frames)",
           "value": round(frames / elapsed, 1), "unit": "frames/s",
           "ms_per_step": round(elapsed / args.steps * 1e3, 3),
           "album": {"tracks": args.tracks * world, "gain_db": album_gain,
                     "peak": album_peak,
                     "collective": "all_reduce SUM uint32[12000] + MAX f64 (RCCL)"
                                   if world > 1 else "none (1 rank)"},
           "bound": "serial fp64 IIR per channel (lane per track-channel, 32 waves)"}
    return out, res, host


def main(argv=None):
    args = parse_args(argv)
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
    device = torch.device("cuda", local)
    os.environ["ATG_DEVICE"] = str(local)

    from audiotools import _atgpu
    eng = _atgpu.Engine(local)
    opts = _atgpu.make_options(**FLAC8)

    n_samples = args.frames * BLOCK
    ids = shard(world, rank, args.tracks)
    pcm = synth_batch(torch, ids, n_samples, device)
    tracks = [(i * n_samples, n_samples) for i in range(args.tracks)]
    n_frames, out_cap = eng.bounds(opts, tracks, 2, 16)
    table = _atgpu.TrackTable(tracks)
    out = torch.empty(out_cap, dtype=torch.uint8, device=device)
    torch.cuda.synchronize()

    def step():
        return eng.encode_device(opts, pcm.data_ptr(), _atgpu.PCM_S16, table, 2, 16,
                                 44100, out.data_ptr(), out_cap)

    for _ in range(args.warmup):
        res = step()

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    kt_sum = {}
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res = step()
        for k, v in eng.kernel_times().items():
            kt_sum[k] = kt_sum.get(k, 0.0) + v
    barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        elapsed = reduce_max(torch, dist, elapsed, device)
    kt = {k: v / args.steps for k, v in kt_sum.items()}
    out_bytes = sum(int(r.bytes) for r in res)
    header = 4 + 4 + 34 + 4 + 4 + 29 + 4 + 4 + 4096
    frame_bytes = out_bytes - header * len(res)

    verified = None
    if not args.no_verify:
        # parity spot check outside the timed region: a few tracks vs oracle
        import oracle_port
        host_out = out.cpu().numpy()
        host_pcm = pcm[:4 * n_samples * 2].cpu().numpy()
        verified = True
        for t in range(min(4, args.tracks)):
            r = res[t]
            img = host_out[r.out_offset:r.out_offset + r.bytes].tobytes()
            want, _ = oracle_port.encode(
                host_pcm[t * n_samples * 2:(t + 1) * n_samples * 2].astype(np.int32),
                2, 16, 44100, **FLAC8)
            verified = verified and (img == want)

    decode = None
    if not args.no_decode:
        decode = decode_leg(args, torch, dist, world, device, out, res, header, n_frames,
                            barrier)

    convert = None
    if not args.no_decode and rank == 0:
        convert = convert_leg(args, torch, device, pcm)
    rg = rg_res = rg_host = None
    if not args.no_decode:
        rg, rg_res, rg_host = replaygain_leg(args, torch, dist, world, rank, device, pcm,
                                             barrier)

    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return

    total_frames = n_frames * world * args.steps
    value = total_frames / elapsed
    # dominant kernel and its roofline.  Algorithmic bytes per launch
    # (DESIGN.md section 4): every kernel that reads the batch reads its
    # PCM once (16,384 B per 4096-sample stereo frame); the packer also
    # writes the compressed frames.
    pcm_bytes = args.tracks * n_samples * 2 * 2
    alg = {"lpc_analyze": pcm_bytes, "subframe_search": pcm_bytes,
           "frame_pack": pcm_bytes + frame_bytes, "track_md5": pcm_bytes,
           "frame_decide": 0, "track_scan": 0, "stream_header": out_bytes - frame_bytes}
    kernels = {k: v for k, v in kt.items() if k != "total"}
    dom = max(kernels, key=kernels.get)
    dom_ms = kernels[dom]
    alg_bytes = alg.get(dom, pcm_bytes)
    achieved = alg_bytes / (dom_ms / 1e3) / 1e9
    traffic = None
    tf = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(tf):
        try:
            traffic = json.load(open(tf)).get(dom)
        except Exception:
            traffic = None

    cpu = None
    if not args.no_cpu_baseline:
        threads = args.cpu_threads or min(16, os.cpu_count() or 1)
        nt = min(args.cpu_sample_tracks, args.tracks)
        sample_frames = args.frames
        sps = sample_frames * BLOCK
        host = pcm.reshape(args.tracks, n_samples * 2)[:nt, :sps * 2].cpu().numpy().reshape(-1)
        fps, dt = cpu_baseline(host, nt, sps, threads)
        cpu = {"value": round(fps, 2), "unit": "frames/s", "cores": threads, "kind": "port",
               "sample": "%d tracks x %d FLAC-8 frames of the same synthetic batch, "
                         "%d threads (one track per thread), %.1f s" % (nt, sample_frames,
                                                                        threads, dt)}
        if rg is not None:
            # oracle on the first 4 tracks: exact title gains/peaks, timed
            import oracle_port
            t0 = time.perf_counter()
            ok = True
            for t in range(min(4, args.tracks)):
                A, pk = oracle_port.rg_title(
                    rg_host[t * n_samples * 2:(t + 1) * n_samples * 2], 2, 16, 44100)
                ok = ok and oracle_port.rg_gain(A) == rg_res[t].title_gain and \
                    pk == rg_res[t].title_peak
            dt = time.perf_counter() - t0
            rg["verified_vs_oracle"] = ok
            rg["cpu_baseline"] = {"value": round(min(4, args.tracks) * args.frames / dt, 2),
                                  "unit": "frames/s", "cores": 1, "kind": "port",
                                  "sample": "oracle title analysis of 4 tracks, 1 thread, "
                                            "%.1f s" % dt}
        if decode is not None:
            host_out = out.cpu().numpy()
            imgs = [host_out[r.out_offset:r.out_offset + r.bytes].tobytes()
                    for r in res[:nt]]
            dfps, ddt = cpu_decode_baseline(imgs, threads)
            decode["cpu_baseline"] = {
                "value": round(dfps, 2), "unit": "frames/s", "cores": threads,
                "kind": "port",
                "sample": "oracle decode of %d of the encoded tracks, %d threads, %.1f s"
                          % (nt, threads, ddt)}

    line = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int32 residuals / f64 LPC analysis (s16 PCM in)",
        "data": "synthetic (seeded sine+noise, 5% white noise, 2% silent tracks)",
        "config": {"workload": "FLAC-8 batch encode, %d tracks x %d frames x 4096 samples "
                               "per GPU, 44.1 kHz 16-bit stereo, PCM and .flac images in HBM"
                               % (args.tracks, args.frames),
                   "tracks_per_gpu": args.tracks, "frames_per_track": args.frames,
                   "block_size": 4096, "preset": "FLAC-8 (-l 12 -m -e -R 6)",
                   "parallelism": "dp%d (tracks sharded per GPU)" % world},
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 2),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                     "alg_bytes_per_launch": alg_bytes, "launch_ms": round(dom_ms, 4)},
        "kernel_ms": {k: round(v, 4) for k, v in kt.items()},
        "compressed_bytes_per_frame": round(frame_bytes / n_frames, 1),
        "verified_vs_oracle": verified,
        "cpu_baseline": cpu,
        "decode": decode,
        "convert": convert,
        "replaygain": rg,
    }
    print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
