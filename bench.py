#!/usr/bin/env python3
"""bench.py — FLAC-8 batch encode throughput on MI355X (BASELINE.json config 2).

One step = one pass of the hot path over one batch: FLAC-8 encode of the
rank's synthetic 44.1 kHz / 16-bit stereo tracks x `--frames` FLAC frames
of 4096 PCM frames, PCM resident in HBM, complete .flac images (STREAMINFO
with MD5, VORBIS_COMMENT, PADDING, frames) left in HBM.

Multi-GPU: one process per GPU.  Under torchrun the ranks come from the
environment; `python bench.py --gpus N` without it spawns the N rank
processes itself before anything touches a GPU.  Tracks are independent, so
ranks share nothing on the data path:
  --scaling weak   (default) every rank encodes `--tracks` tracks of its own;
  --scaling strong the `--tracks` tracks are split over the ranks.
value = frames of all ranks / max-over-ranks time of the K timed steps.

Prints ONE JSON line on rank 0.  Parity: every GPU image of the batch is
byte-compared with the CPU port (oracle/flac_port.c, pinned to the reference)
and a sample with the reference encoder itself (oracle/_ref/flacenc, built
from the reference's own C sources) when that build is present; the decode
leg compares every decoded sample with the source PCM.  `roofline` is the
HBM roofline of the longest kernel on the critical (main-stream) path,
`roofline_valu` its integer-VALU roofline, `step_hbm` the whole step's
algorithmic HBM fraction.  cpu_baseline = the reference encoder on this
host's cores (one process per track, like track2track -j N).
"""
import argparse
import json
import os
import socket
import struct
import subprocess
import sys
import queue
import tempfile
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
F64_PEAK_TFLOPS = 78.6         # MI355X FP64 vector, AMD spec (= half the 157.3 TF FP32 vector
                               # peak of MI355X_MICROARCH.md; the guide lists no f64 row)
# integer VALU issue peak: 256 CUs x 4 SIMDs, one wave64 VALU instruction
# per 2 cycles per SIMD (MI355X_MICROARCH.md "Wave scheduling"), 2.4 GHz
N_SIMD = 1024
CLOCK_HZ = 2.4e9
VALU_PEAK_WAVE_INSTS = N_SIMD * CLOCK_HZ / 2.0
FLAC8 = dict(block_size=4096, max_lpc_order=12, min_residual_partition_order=0,
             max_residual_partition_order=6, mid_side=True,
             exhaustive_model_search=True)
HEADER_BYTES = 4 + 4 + 34 + 4 + 4 + 29 + 4 + 4 + 4096
# kernels on the encoder's main stream, in launch order (MD5 runs on its own
# stream beside them, engine.hip)
MAIN_STREAM = ("subframe_search", "frame_decide", "track_scan", "frame_pack")


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--inflight", type=int, default=12,
                    help="encode batches in flight (2..32; from 4 on the MD5 chains are "
                         "rolled, atg_engine_set_inflight)")
    ap.add_argument("--tracks", type=int, default=1024,
                    help="tracks per GPU (weak) or in total (strong)")
    ap.add_argument("--frames", type=int, default=64, help="FLAC frames per track")
    ap.add_argument("--scaling", choices=("weak", "strong"), default="weak")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--cpu-ref-tracks", type=int, default=256,
                    help="tracks the reference encoder baseline encodes")
    ap.add_argument("--narrow", default="512,256,128",
                    help="track counts of the narrow-batch leg (a strong-scaling rank's "
                         "share, on one GPU); empty to skip")
    ap.add_argument("--narrow-depths", default="auto,3,32",
                    help="batches in flight for the narrow leg (atg_engine_set_inflight; "
                         "auto = the engine's automatic depth)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--chain-tracks", type=int, default=64,
                    help="config-5 chain leg: 192 kHz 5.1 tracks per GPU")
    ap.add_argument("--chain-seconds", type=int, default=10)
    ap.add_argument("--chain-inflight", type=int, default=3,
                    help="config-5 chain leg: FLAC batches in flight (3: 31.7-32.0 ms per "
                         "step, 4: 33.0-33.1, 5-6 slower; with the MD5 on the host no "
                         "GPU chains need hiding; from 4 on GPU chains are rolled)")
    ap.add_argument("--chain-decoders", type=int, default=3,
                    help="config-5 chain leg: ALAC decoders (PCM buffers) each decode thread "
                         "cycles through")
    ap.add_argument("--chain-decode-threads", type=int, default=1,
                    help="config-5 chain leg: decode threads, batch k on thread k mod T (T "
                         "decodes at once; 2 and 3 measured 34.7-35.1 and 32.9 ms per step "
                         "against 33.4 for 1: the device is already full)")
    ap.add_argument("--chain-md5", choices=("auto", "gpu", "host"), default="auto",
                    help="config-5 chain leg: where the FLAC batches' MD5 runs (the engine's "
                         "choice, rolled GPU chains, or host threads)")
    ap.add_argument("--no-chain", action="store_true")
    ap.add_argument("--no-host", action="store_true", help="skip the host-to-host leg")
    ap.add_argument("--no-t2t", action="store_true", help="skip the track2track leg")
    ap.add_argument("--t2t-procs", type=int, default=8,
                    help="track2track leg: conversion processes alive at a time (-j)")
    ap.add_argument("--t2t-files", type=int, default=128,
                    help="track2track leg: 64-frame WAV files, one process each")
    ap.add_argument("--no-rg4", action="store_true", help="skip the config-4 ReplayGain leg")
    ap.add_argument("--rg4-seconds", type=int, default=10)
    ap.add_argument("--dec-inflight", type=int, default=12,
                    help="decode batches in flight (the decoder's slot count, 3..16; from 4 "
                         "on the MD5 hashes are rolled, atg_decoder_set_inflight; 12 measured "
                         "7.03-7.05 ms per step against 7.16-7.23 at 8, 7.08 at 10 and 8.33 "
                         "at 16, profiles/r05_zz_dec_depth.txt)")
    ap.add_argument("--dec-hypothesis", type=int, default=1, choices=(0, 1, 2),
                    help="the decoder's frame-end hypothesis (atg_decoder_set_frame_hypothesis):"
                         " 0 every subframe walked by the parse, 1 (default), 2 every batch "
                         "redone (self-check)")
    ap.add_argument("--no-decode", action="store_true",
                    help="skip the decode / convert / ReplayGain legs")
    ap.add_argument("--k2-profile", action="store_true",
                    help="only the headline batch's search kernel, one batch at a time "
                         "(for rocprofv3 --kernel-trace --stats; prints a line that is not "
                         "a measurement)")
    ap.add_argument("--selftest", action="store_true",
                    help="harness self-test on CPU (gloo, oracle as the step); "
                         "prints a line that is not a measurement")
    return ap.parse_args(argv)


def shard(n_total_ranks, rank, tracks, scaling="weak"):
    """global track ids owned by `rank`.  weak: a full batch of `tracks` per
    rank; strong: `tracks` split into contiguous near-equal slices.  Tracks
    are independent, so ranks share nothing on the data path."""
    if scaling == "weak":
        return list(range(rank * tracks, (rank + 1) * tracks))
    lo = rank * tracks // n_total_ranks
    hi = (rank + 1) * tracks // n_total_ranks
    return list(range(lo, hi))


def reduce_max(torch, dist, value, device):
    """max of a host float over all ranks (the step clock: max over ranks)"""
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def reduce_sum(torch, dist, value, device):
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch(args, argv):
    """spawn one rank process per GPU (this process never touches a GPU);
    returns the worst exit code"""
    port = _free_port()
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv,
                                      env=env))
    rc = 0
    for p in procs:
        rc = max(rc, abs(p.wait()))
    return rc


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
    gen.manual_seed(0x5EED + (track_ids[0] if track_ids else 0))
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


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_share():
    """host CPUs this process may use: the affinity mask, the cgroup CPU
    quota and the harness's stated share (OMP_NUM_THREADS is set to the
    box's per-GPU CPU share) -> (threads to use, details)"""
    info = {"os_cpu_count": os.cpu_count()}
    n = os.cpu_count() or 1
    try:
        info["affinity"] = len(os.sched_getaffinity(0))
        n = min(n, info["affinity"])
    except (AttributeError, OSError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            info["cgroup_quota_cpus"] = round(int(q) / int(per), 2)
            n = min(n, max(1, int(int(q) // int(per))))
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit():
        info["omp_num_threads"] = int(omp)
        n = min(n, int(omp))
    info["used"] = n
    return n, info


def _parallel(n_items, threads, fn):
    """run fn(i) for i < n_items on `threads` host threads (the work is
    ctypes / subprocess calls, which release the GIL); -> seconds"""
    work = list(range(n_items - 1, -1, -1))
    lock = threading.Lock()
    err = []

    def run():
        while True:
            with lock:
                if not work or err:
                    return
                i = work.pop()
            try:
                fn(i)
            except Exception as e:  # surfaced after join
                with lock:
                    err.append(e)

    th = [threading.Thread(target=run) for _ in range(max(1, threads))]
    t0 = time.perf_counter()
    for x in th:
        x.start()
    for x in th:
        x.join()
    if err:
        raise err[0]
    return time.perf_counter() - t0


def port_encode_all(pcm_host, n_tracks, samples_per_track, threads):
    """the CPU port (oracle/flac_port.c) encodes every track of the batch on
    `threads` host threads, one track per thread at a time like
    track2track -j N; -> (images, seconds)"""
    import oracle_port
    oracle_port.load()
    images = [None] * n_tracks

    def one(t):
        p = pcm_host[t * samples_per_track * 2:(t + 1) * samples_per_track * 2]
        images[t], _ = oracle_port.encode(p.astype(np.int32), 2, 16, 44100, **FLAC8)

    return images, _parallel(n_tracks, threads, one)


def ref_encode_sample(pcm_host, n_tracks, samples_per_track, procs):
    """the reference encoder itself (oracle/_ref/flacenc = the reference's
    src/encoders/flac.c built standalone from its own sources), one process
    per track, `procs` at a time; -> (images, seconds) or None when the
    build is absent"""
    import oracle_port
    exe = oracle_port.REF_FLACENC
    if not os.path.exists(exe):
        return None
    args = [exe, "-c", "2", "-r", "44100", "-b", "16", "-B", "4096", "-l", "12", "-P", "0",
            "-R", "6", "-m", "-e"]
    images = [None] * n_tracks
    raws = [pcm_host[t * samples_per_track * 2:(t + 1) * samples_per_track * 2]
            .astype("<i2").tobytes() for t in range(n_tracks)]
    with tempfile.TemporaryDirectory() as d:
        def one(t):
            fn = os.path.join(d, "%d.flac" % t)
            subprocess.run(args + [fn], input=raws[t], stdout=subprocess.DEVNULL, check=True)
            with open(fn, "rb") as f:
                images[t] = f.read()

        dt = _parallel(n_tracks, procs, one)
    return images, dt


def load_profile_json(name):
    fn = os.path.join(ROOT, "profiles", name)
    if os.path.exists(fn):
        try:
            with open(fn) as f:
                return json.load(f)
        except (OSError, ValueError):
            return None
    return None


def decode_leg(args, torch, dist, world, device, eng, out, res, pcm, pcm_host, n_frames,
               barrier):
    """GPU decode of the batch the encoder just left in HBM (the trackverify
    path): every track decoded, its STREAMINFO MD5
    checked on the GPU, and every decoded sample compared with the source
    PCM (lossless round trip).  Returns the JSON object."""
    from audiotools import _atgpu
    dec = _atgpu.Decoder(int(os.environ.get("LOCAL_RANK", "0")))
    if args.dec_inflight > 3:
        # rolled MD5 hashes (atg_decoder_set_inflight)
        dec.set_inflight(args.dec_inflight)
    if args.dec_hypothesis != 1:
        dec.set_frame_hypothesis(args.dec_hypothesis)
    tracks = []
    for r in res:
        si = _atgpu.StreamInfo()
        si.total_samples = args.frames * BLOCK
        si.sample_rate, si.channels, si.bits_per_sample = 44100, 2, 16
        si.max_block_size = BLOCK
        si.md5[:] = bytes(r.md5)
        tracks.append(_atgpu.dec_track(r.out_offset + HEADER_BYTES, r.bytes - HEADER_BYTES, si))
    nbytes = max(r.out_offset + r.bytes for r in res)

    kt_sum = {}

    def run(k_steps, timed):
        # dec_inflight batches in flight (atg_flac_decode_device_async):
        # batch k's restore and emit run under batch k+1's scan and parse,
        # its MD5 hashes rolled over the batches behind it from 4 in flight
        # on; every batch is waited (drained) inside the timed region
        pending, last = [], None

        def wait_one():
            r = dec.decode_wait(pending.pop(0))
            if timed:
                for k, v in dec.kernel_times().items():
                    kt_sum[k] = kt_sum.get(k, 0.0) + v
            return r

        for _ in range(k_steps):
            if len(pending) == args.dec_inflight:
                last = wait_one()
            pending.append(dec.decode_device_async(out.data_ptr(), nbytes, tracks))
        while pending:
            last = wait_one()
        return last

    # untimed warm-up: every slot of the rotation (each slot's ~5 GB of PCM
    # rows, PCM and MD5 bytes are allocated on its first batch), then on to
    # ~40 batches -- in a process whose engine ran host jobs just before, the
    # first ~40 rolled batches ran 1.5-2 ms per step slower, the MD5 slices
    # falling behind
    run(max(args.warmup, 5 * args.dec_inflight), False)
    barrier()
    t0 = time.perf_counter()
    dres, d_pcm, nsamp = run(args.steps, True)
    barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        elapsed = reduce_max(torch, dist, elapsed, device)
    kt = {k: v / args.steps for k, v in kt_sum.items()}
    ok = all(r.status == 0 and r.pcm_frames == args.frames * BLOCK for r in dres)
    # every decoded sample vs the source PCM (exact), outside the timed region
    same = False
    if ok and nsamp == pcm.numel():
        got = np.empty(int(nsamp), dtype=np.int32)
        eng.copy_to_host(got, d_pcm)
        same = bool(np.array_equal(got, pcm_host))
        del got
    comp = sum(int(r.bytes) - HEADER_BYTES for r in res)
    pcm32 = len(res) * args.frames * BLOCK * 2 * 4
    # algorithmic bytes per launch: the parsers read the compressed frames
    # once; the subframe decoder also writes its int32 row scratch, which
    # the emitter reads, writing int32 PCM + the s16 byte stream
    alg = {"dec_scan": comp, "dec_parse": comp, "dec_chain": 0,
           "dec_subframe": comp + pcm32, "dec_emit": pcm32 * 2 + pcm32 // 2,
           "dec_md5": pcm32 // 2}
    # the dominant kernel on the critical path: the MD5 chains run beside the
    # next batch on their own stream
    kernels = {k: v for k, v in kt.items() if k in alg and k != "dec_md5"}
    dom = max(kernels, key=kernels.get)
    achieved = alg[dom] / (kernels[dom] / 1e3) / 1e9
    traffic = (load_profile_json("pmc_traffic.json") or {}).get(dom)
    redos = dec.frame_hypothesis_redos()
    dec.close()
    step_alg = comp + pcm32
    return {
        "metric": "FLAC-8 decode frames/s (GPU decode of the encoded batch, MD5-verified)",
        "value": round(n_frames * world * args.steps / elapsed, 1), "unit": "frames/s",
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "kernel_ms": {k: round(v, 4) for k, v in kt.items()},
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 2),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                     "alg_bytes_per_launch": alg[dom], "launch_ms": round(kernels[dom], 4),
                     "selection": "longest kernel on the decoder (critical-path) stream"},
        "pipelining": ("%d batches in flight: restore, emit and MD5 of batch k on its slot's "
                       "stream beside the scan and parse of batch k+1" % args.dec_inflight)
                      if args.dec_inflight <= 3 else
                      ("%d batches in flight: restore and emit beside the next batch's scan and "
                       "parse, every batch's MD5 hashes advanced together in %d slices (rolled)"
                       % (args.dec_inflight, args.dec_inflight - 2)),
        "step_hbm": {"alg_bytes_per_step": step_alg,
                     "frac": round(step_alg / (elapsed / args.steps) / 1e9 / HBM_PEAK_GBS, 5)},
        "frame_hypothesis": {"mode": args.dec_hypothesis, "batches_redone": redos,
                             "note": "the parse takes a frame's end from the next header "
                                     "candidate with a zero CRC-16 residue and skips the "
                                     "frame's last subframe; the restore checks it, a failed "
                                     "check redoes the batch with the full parse"},
        "verified_md5_round_trip": ok,
        "verified_pcm_vs_source": same,
        "verified_tracks": len(dres) if (ok and same) else 0,
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
    traffic = (load_profile_json("pmc_traffic.json") or {}).get("pcm_bps")
    return {"metric": "BPSConverter 16->8 dither, samples/s", "value": round(frames * 2 / dt, 1),
            "unit": "samples/s", "ms_per_step": round(dt * 1e3, 4),
            "roofline": {"bound": "hbm", "kernel": "k_pcm_bps",
                         "achieved": round(alg / dt / 1e9, 2), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(alg / dt / 1e9 / HBM_PEAK_GBS, 4),
                         "traffic": traffic, "alg_bytes_per_launch": alg,
                         "launch_ms": round(dt * 1e3, 4)},
            "verified_dither_invariant": ok}


def host_leg(args, torch, dist, world, device, eng, opts, pcm_host, tracks, n_frames, images,
             barrier):
    """SURVEY 8(d)'s host-to-host timer: host PCM in, .flac images back in
    host memory, through the chunked pipeline of atg_flac_encode_host_async
    -- chunks of ~512 MB of PCM, three in flight (chunk c+1's upload, chunk
    c's encode and chunk c-1's download overlap), each chunk's MD5 chains
    from the moment its PCM is on the device, images packed on the device
    and copied back in one transfer per chunk.  Batches are queued back to
    back (three jobs in flight, three output buffers), so batch k+1's uploads
    overlap batch k's last chunks.  The headline form keeps PCM and output
    in pinned host memory, as 8(d) specifies (DMA straight from / to them);
    a synchronous call per batch and the pageable form (numpy buffers,
    staged through pinned memory on 16 host threads) are reported beside
    it.  Every image is compared with the device-path image of the same
    track."""
    from audiotools import _atgpu
    # up to 20 batches: the pipeline's fill (the first upload) and drain
    # (the last batch's MD5 chains and download) are inside the clock
    steps = max(2, min(args.steps, 20))
    nb = eng.bounds(opts, tracks, 2, 16)[1]
    pin_pcm = _atgpu.pinned_empty(pcm_host.shape, np.int16)
    pin_pcm[:] = pcm_host
    pin_outs = [_atgpu.pinned_empty(nb, np.uint8) for _ in range(3)]
    in_b = pcm_host.nbytes

    def check(o, res):
        return all(bytes(o[r.out_offset:r.out_offset + r.bytes]) == images[t]
                   for t, r in enumerate(res))

    def summary(elapsed, n, o, res, same):
        if world > 1:
            elapsed = reduce_max(torch, dist, elapsed, device)
        out_b = sum(int(r.bytes) for r in res)
        ms = elapsed / n * 1e3
        return {"value": round(n_frames * world * n / elapsed, 1), "unit": "frames/s",
                "ms_per_step": round(ms, 3), "steps": n,
                "bytes_in": in_b, "bytes_out": out_b,
                "pcie_gbps": round((in_b + out_b) / (ms / 1e3) / 1e9, 2),
                "images_identical_to_device_path": same}

    def run_async(pcm, outs):
        eng.encode(opts, pcm, tracks, 2, 16, 44100, out=outs[0])  # warm-up
        barrier()
        t0 = time.perf_counter()
        pend, last = [], None
        for k in range(steps):
            pend.append(eng.encode_async(opts, pcm, tracks, 2, 16, 44100, out=outs[k % 3]))
            if len(pend) > 2:
                last = pend.pop(0).wait()
        while pend:
            last = pend.pop(0).wait()
        barrier()
        elapsed = time.perf_counter() - t0
        return summary(elapsed, steps, last[0], last[1], check(last[0], last[1]))

    def run_sync(pcm, out):
        eng.encode(opts, pcm, tracks, 2, 16, 44100, out=out)  # warm-up
        barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            o, res, _, _ = eng.encode(opts, pcm, tracks, 2, 16, 44100, out=out)
        barrier()
        elapsed = time.perf_counter() - t0
        return summary(elapsed, steps, o, res, check(o, res))

    chunk_mb = int(os.environ.get("ATG_BENCH_HOST_CHUNK_MB", "512"))
    if chunk_mb != 512:
        eng.set_host_chunk_bytes(chunk_mb << 20)
    pinned = run_async(pin_pcm, pin_outs)
    sync = run_sync(pin_pcm, pin_outs[0])
    pageable = run_sync(pcm_host, None)
    if chunk_mb != 512:
        eng.set_host_chunk_bytes(512 << 20)
    del pin_pcm, pin_outs
    out = {"metric": "FLAC-8 encode frames/s, host PCM in -> .flac images in host memory "
                     "(pinned buffers, batches queued back to back, SURVEY 8(d) timer)"}
    out.update(pinned)
    out["chunk_mb"] = chunk_mb
    out["sync_per_batch"] = sync
    out["pageable_sync"] = pageable
    return out


def resample_leg(args, torch, dist, world, device, pcm, n_tracks, barrier, threads, verify):
    """BASELINE config 3: 44.1 kHz -> 48 kHz sinc resample (resample.hip,
    SURVEY 8(a) R1-R3) + 24 -> 16-bit dither (pcm_convert.hip R4) of every
    track of the batch, 24-bit stereo in HBM.  Every resampled sample of
    every track is compared with the CPU restatement oracle/resample_port.c
    (parity unpinned to reference output: BEST table absent), outside the
    timed region.  Returns the JSON object."""
    from audiotools import _atgpu
    lib = _atgpu.load_library()
    n_in = args.frames * BLOCK
    x16 = pcm.to(torch.int32)
    x = x16 * 256 + ((x16 * 73 + 41) & 255)  # 24-bit: the signal plus low bits
    del x16
    tracks = [(t * n_in, n_in, 44100, 48000) for t in range(n_tracks)]
    n_out = _atgpu.resample_output_frames(n_in, 2, 44100, 48000)
    total = n_out * n_tracks
    y = torch.empty(total * 2, dtype=torch.int32, device=device)
    z = torch.empty_like(y)
    dither = torch.randint(0, 256, ((total * 2 + 7) // 8,), dtype=torch.uint8, device=device)
    stream = torch.cuda.current_stream(device).cuda_stream
    torch.cuda.synchronize()

    def step():
        _atgpu.resample_device(x.data_ptr(), y.data_ptr(), total * 2, tracks, 2, 24, stream)
        st = lib.atg_pcm_convert_device(_atgpu.CONV_BPS, y.data_ptr(), z.data_ptr(), total, 2,
                                        0, 24, 16, dither.data_ptr(), 0, stream)
        if st != _atgpu.ATG_OK:
            raise RuntimeError(lib.atg_pcm_convert_last_error())

    for _ in range(args.warmup):
        step()
    kt_sum = {}
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        for k, v in _atgpu.resample_kernel_times().items():
            kt_sum[k] = kt_sum.get(k, 0.0) + v
    barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        elapsed = reduce_max(torch, dist, elapsed, device)
    kt = {k: v / args.steps for k, v in kt_sum.items()}
    dither_ok = bool((((z ^ (y >> 8)) & ~1) == 0).all().item())
    # fp64 roofline of the filter: the reference's arithmetic per output
    # frame is (taps) x (2 flops to interpolate the coefficient + 2 per
    # channel to accumulate); taps = 2 x half_len x 4096 / increment on
    # average (45.70 per side at 44.1k -> 48k)
    taps = 2.0 * 22437 * 4096 / (491 * 4096)
    flops = total * taps * (2 + 2 * 2)
    f_ms = kt.get("rs_filter", 0.0)
    achieved = flops / (f_ms / 1e3) / 1e12 if f_ms else None
    hbm = (n_tracks * n_in + total) * 2 * 4
    out = {"metric": "44.1k->48k sinc resample + 24->16 dither, output frames/s (config 3)",
           "value": round(total * world * args.steps / elapsed, 1), "unit": "frames/s",
           "ms_per_step": round(elapsed / args.steps * 1e3, 3),
           "realtime_x": round(n_tracks * world * n_in / 44100.0 / (elapsed / args.steps), 1),
           "config": {"tracks_per_gpu": n_tracks, "input_frames_per_track": n_in,
                      "output_frames_per_track": n_out, "channels": 2, "bits": "24 -> 16",
                      "coefficients": "libsamplerate MEDIUM (BEST table absent from the "
                                      "reference tree)"},
           "kernel_ms": {k: round(v, 4) for k, v in kt.items()},
           "roofline": {"bound": "f64-valu", "kernel": "rs_filter",
                        "achieved": round(achieved, 3) if achieved else None,
                        "peak": F64_PEAK_TFLOPS, "unit": "TFLOP/s",
                        "frac": round(achieved / F64_PEAK_TFLOPS, 4) if achieved else None,
                        "alg_flops_per_launch": flops, "launch_ms": round(f_ms, 4),
                        # the reference rounds each product (no FMA): a tap is a
                        # v_mul_f64 + v_add_f64 pair, so the attainable rate is
                        # half the FMA peak
                        "peak_no_fma": F64_PEAK_TFLOPS / 2,
                        "frac_no_fma": round(achieved / (F64_PEAK_TFLOPS / 2), 4)
                        if achieved else None,
                        "hbm_alg_bytes": hbm,
                        "hbm_frac": round(hbm / (f_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4)
                        if f_ms else None},
           "verified_dither_invariant": dither_ok}
    if verify:
        import oracle_port
        oracle_port.load()
        yh = y.cpu().numpy()
        xh = x.cpu().numpy()
        bad = []

        def one(t):
            want = oracle_port.resample(xh[t * n_in * 2:(t + 1) * n_in * 2], 2, 24,
                                        48000 / 44100.0)
            if not np.array_equal(want, yh[t * n_out * 2:(t + 1) * n_out * 2]):
                bad.append(t)

        dt = _parallel(n_tracks, threads, one)
        out["verified_vs_oracle"] = not bad
        out["verified_tracks"] = n_tracks - len(bad)
        t1 = min(2, n_tracks)
        dt1 = _parallel(t1, 1, one)
        out["cpu_baseline"] = {
            "value": round(t1 * n_out / dt1, 1), "unit": "frames/s", "cores": 1,
            "kind": "port", "sample": "oracle/resample_port.c on %d tracks, 1 thread, %.1f s"
                                      % (t1, dt1),
            "n_threads": {"value": round(n_tracks * n_out / dt, 1), "cores": threads,
                          "sample": "all %d tracks, %d threads, %.1f s"
                                    % (n_tracks, threads, dt)}}
        del yh, xh
    del x, y, z, dither
    return out


def chain_leg(args, torch, dist, world, device, barrier, threads, verify):
    """BASELINE config 5, the track2track chain: ALAC (192 kHz / 24-bit /
    5.1) decode -> 48 kHz sinc resample -> FLAC-8 encode, all three on the
    GPU with the data left in HBM between stages (alac_decode.hip ->
    resample.hip -> the FLAC encoder).  The ALAC input is made once, untimed,
    by the GPU ALAC encoder from synthetic PCM.  Checks outside the timed
    region: every decoded sample equals the source (lossless); the first
    tracks' resampled PCM vs oracle/resample_port.c and FLAC images vs the
    FLAC port, bit for bit."""
    from audiotools import _atgpu
    ch, rin, rout, bps = 6, 192000, 48000, 24
    n_tracks, n_in = args.chain_tracks, args.chain_seconds * rin
    local = int(os.environ.get("LOCAL_RANK", "0"))
    g = torch.Generator(device=device)
    g.manual_seed(11 + int(os.environ.get("RANK", "0")))
    t = torch.arange(n_in, device=device, dtype=torch.float64)
    src = torch.empty((n_tracks, n_in, ch), dtype=torch.int32, device=device)
    for k in range(n_tracks):
        # tone + noise, peaks below 2^23 (a 24-bit source must fit 24 bits to
        # round-trip losslessly)
        f = (110.0 + 37.0 * k + 55.0 * torch.arange(ch, device=device, dtype=torch.float64))
        tone = torch.sin(2 * np.pi * t[:, None] * f[None, :] / rin) * (3e6 + 1e5 * (k % 40))
        noise = torch.randint(-4096, 4096, (n_in, ch), device=device, generator=g,
                              dtype=torch.int32)
        src[k] = tone.to(torch.int32) + noise
    del t
    src = src.reshape(-1)
    # the library's kernels run on their own non-blocking streams: the torch
    # work that produced their inputs must be finished first
    torch.cuda.synchronize()
    # ALAC input (untimed): one mdat atom per track, framesets from the encoder
    aenc = _atgpu.AlacEncoder(local)
    aopts = aenc.options()
    atracks = [(k * n_in, n_in) for k in range(n_tracks)]
    n_fs, acap = aenc.bounds(aopts, atracks, ch, bps)
    alac = torch.zeros(acap, dtype=torch.uint8, device=device)
    fsb = np.zeros(max(1, n_fs), dtype=np.uint32)
    torch.cuda.synchronize()
    ares = aenc.encode_device(aopts, src.data_ptr(), _atgpu.PCM_S32, atracks, ch, bps,
                              alac.data_ptr(), acap, fsb)
    aenc.close()
    if any(r.status for r in ares):
        raise RuntimeError("ALAC encode failed: %s" % sorted({int(r.status) for r in ares}))
    info = _atgpu.AlacInfo()
    info.max_samples_per_frame, info.bits_per_sample = 4096, bps
    info.history_multiplier, info.initial_history, info.maximum_k = 40, 10, 14
    info.channels, info.sample_rate, info.total_frames = ch, rin, n_in
    dtracks = []
    for r in ares:
        dtracks.append(_atgpu.alac_dec_track(
            r.out_offset, r.bytes, info, start=8, remaining=n_in,
            frameset_bytes=fsb[r.first_frameset:r.first_frameset + r.n_framesets]))
    alac_bytes = sum(int(r.bytes) for r in ares)
    nbytes = max(int(r.out_offset + r.bytes) for r in ares)
    # the pipeline: n_thr decode threads run the next
    # batches' ALAC decodes (batch k on thread k mod n_thr), each on n_dec
    # decoders of its own (each owns its PCM buffer; three let a thread run
    # two of its batches ahead), while the main thread resamples batch k and
    # enqueues its FLAC encode; ctypes releases the GIL inside every library
    # call, so the GPU sees the ALAC kernels of n_thr batches beside the
    # resampler's and the encoder's.  A decoder is handed back once the
    # (synchronous) resample has read its buffer.
    n_dec = max(2, args.chain_decoders)
    n_thr = max(1, args.chain_decode_threads)
    adecs = [_atgpu.AlacDecoder(local) for _ in range(n_dec * n_thr)]
    rtracks = [(k * n_in, n_in, rin, rout) for k in range(n_tracks)]
    n_out = _atgpu.resample_output_frames(n_in, ch, rin, rout)
    # `depth` resampled-PCM and FLAC buffers: batch k is waited once batch
    # k + depth - 1 is enqueued; from depth 4 on the encoder rolls every
    # in-flight batch's MD5 chains forward in one launch per enqueue
    # (atg_engine_set_inflight), so the serial per-track hashes (~9 MB per
    # 5.1 track) stay off the step's critical path
    depth = max(3, args.chain_inflight)
    ys = [torch.empty(n_out * n_tracks * ch, dtype=torch.int32, device=device)
          for _ in range(depth)]
    eng = _atgpu.Engine(local, md5=args.chain_md5)
    eng.set_inflight(depth)
    fopts = _atgpu.make_options(**FLAC8)
    ftracks = [(k * n_out, n_out) for k in range(n_tracks)]
    n_flac, fcap = eng.bounds(fopts, ftracks, ch, bps)
    ftable = _atgpu.TrackTable(ftracks)
    flacs = [torch.empty(fcap, dtype=torch.uint8, device=device) for _ in range(depth)]
    rs_stream = torch.cuda.Stream(device)
    stream = rs_stream.cuda_stream
    state = {}
    pending = []
    kt = {}

    torch.cuda.synchronize()

    def decode_thread(ks, free, ready):
        try:
            for k in ks:
                i = free.get()
                if i is None:  # the main thread gave up
                    return
                dres, d_pcm, nsamp = adecs[i].decode_device(alac.data_ptr(), nbytes, dtracks)
                ready.put((k, i, dres, d_pcm, nsamp))
        except BaseException as e:  # re-raised on the main thread
            ready.put(e)

    def run(first, count, timed):
        frees = [queue.Queue() for _ in range(n_thr)]
        readies = [queue.Queue() for _ in range(n_thr)]
        for j in range(n_thr):
            for i in range(j * n_dec, (j + 1) * n_dec):
                frees[j].put(i)
        ths = [threading.Thread(target=decode_thread,
                                args=(range(first + j, first + count, n_thr), frees[j],
                                      readies[j]), daemon=True) for j in range(n_thr)]
        for th in ths:
            th.start()
        try:
            for kk in range(count):
                item = readies[kk % n_thr].get()
                if isinstance(item, BaseException):
                    raise item
                k, i, dres, d_pcm, nsamp = item
                free = frees[kk % n_thr]
                # the resampler reads n_in frames per track at fixed offsets:
                # only a complete decode may feed it
                if nsamp != src.numel() or any(r.status or r.pcm_frames != n_in for r in dres):
                    raise RuntimeError("ALAC decode incomplete: %d samples, statuses %s"
                                       % (nsamp, sorted({int(r.status) for r in dres})))
                y = ys[k % depth]
                _atgpu.resample_device(d_pcm, y.data_ptr(), y.numel(), rtracks, ch, bps, stream)
                if timed:
                    for pre, d in (("alac_", adecs[i].kernel_times()),
                                   ("", _atgpu.resample_kernel_times())):
                        for name, v in d.items():
                            key = name if name.startswith(pre) else pre + name
                            kt[key] = kt.get(key, 0.0) + v / args.steps
                if k == first + count - 1:
                    state.update(dres=dres, d_pcm=d_pcm, nsamp=nsamp, last=k)
                else:
                    free.put(i)
                pending.append(eng.encode_device_async(
                    fopts, y.data_ptr(), _atgpu.PCM_S32, ftable, ch, bps, rout,
                    flacs[k % depth].data_ptr(), fcap))
                if len(pending) >= depth:
                    state["fres"] = eng.wait(pending.pop(0))
                    if timed:
                        for name, v in eng.kernel_times().items():
                            key = name if name.startswith("flac_") else "flac_" + name
                            kt[key] = kt.get(key, 0.0) + v / args.steps
            while pending:
                state["fres"] = eng.wait(pending.pop(0))
                if timed:
                    for name, v in eng.kernel_times().items():
                        key = name if name.startswith("flac_") else "flac_" + name
                        kt[key] = kt.get(key, 0.0) + v / args.steps
        finally:
            for f in frees:
                f.put(None)  # a thread still waiting for a decoder stops
            for th in ths:
                th.join()

    if args.warmup:
        run(0, args.warmup, False)
    barrier()
    t0 = time.perf_counter()
    run(args.warmup, args.steps, True)
    barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        elapsed = reduce_max(torch, dist, elapsed, device)
    last = args.warmup + args.steps - 1
    y = ys[last % depth]
    flac = flacs[last % depth]
    dres, fres = state["dres"], state["fres"]
    dec_ok = all(r.status == 0 and r.pcm_frames == n_in for r in dres) and \
        state["nsamp"] == src.numel()
    lossless, bad_track = _device_equal(torch, eng, state["d_pcm"], src, n_tracks) if dec_ok \
        else (False, -3)
    flac_bytes = sum(int(r.bytes) for r in fres)
    out = {"metric": "config 5 track2track chain: ALAC 192k/24-bit 5.1 decode -> 48k resample "
                     "-> FLAC-8, output frames/s (48 kHz PCM frames)",
           "value": round(n_out * n_tracks * world * args.steps / elapsed, 1),
           "unit": "frames/s", "ms_per_step": round(elapsed / args.steps * 1e3, 3),
           "flac_frames_per_s": round(n_flac * world * args.steps / elapsed, 1),
           "realtime_x": round(n_tracks * world * args.chain_seconds / (elapsed / args.steps), 1),
           "config": {"tracks_per_gpu": n_tracks, "seconds_per_track": args.chain_seconds,
                      "channels": ch, "bits": bps, "rates": "%d -> %d" % (rin, rout),
                      "alac_bytes": alac_bytes, "flac_bytes": flac_bytes,
                      "flac_frames": n_flac,
                      "pipeline": "%d decode threads (%d ALAC decoders each) beside resample + "
                                  "FLAC encode, %d FLAC batches in flight" % (n_thr, n_dec, depth)},
           "kernel_ms": {k: round(v, 4) for k, v in kt.items()},
           "verified_alac_lossless": bool(dec_ok and lossless),
           "alac_decode_status": sorted({int(r.status) for r in dres}),
           "alac_decode_frames_ok": all(int(r.pcm_frames) == n_in for r in dres),
           "alac_decode_samples": int(state["nsamp"]),
           "alac_first_bad_track": bad_track}
    if verify:
        out.update(chain_verify(args, threads, ch, bps, rin, rout, n_tracks, n_in, n_out, info,
                                ares, fsb, fres, alac, src, y, flac))
    for a in adecs:
        a.close()
    eng.close()
    del src, alac, y, flac, ys, flacs
    return out


def chain_verify(args, threads, ch, bps, rin, rout, n_tracks, n_in, n_out, info, ares, fsb,
                 fres, alac, src, y, flac):
    """config-5 parity outside the timed region, EVERY track: the port
    decodes each GPU-written ALAC track back to the source, resamples it
    (oracle/resample_port.c) and FLAC-8 encodes that (oracle/flac_port.c);
    the GPU's resampled PCM and FLAC image must equal the port's bit for
    bit.  Then the CPU baseline: the reference's own ALAC decoder and FLAC
    encoder (oracle/_ref/alacdec, flacenc) as processes around the resample
    port (the reference's resampler is unbuildable: BEST table absent), one
    track per worker like track2track -j N."""
    import oracle_port
    from audiotools import m4a
    oracle_port.load()
    yh = y.cpu().numpy()
    sh = src.cpu().numpy()
    fh = flac.cpu().numpy()
    alac_h = alac.cpu().numpy()
    ainfo = oracle_port.AlacInfo()
    for f in ("max_samples_per_frame", "bits_per_sample", "history_multiplier",
              "initial_history", "maximum_k", "channels", "sample_rate", "total_frames"):
        setattr(ainfo, f, getattr(info, f))
    bad = {"alac": [], "resample": [], "flac": []}

    def one(k):
        r = ares[k]
        mdat = alac_h[r.out_offset:r.out_offset + r.bytes].tobytes()
        d = oracle_port.alac_decode(mdat, info=ainfo, start=8, remaining=n_in)
        x = sh[k * n_in * ch:(k + 1) * n_in * ch]
        if d["code"] != 0 or not np.array_equal(d["pcm"], x):
            bad["alac"].append(k)
        want = oracle_port.resample(x, ch, bps, rout / rin)
        if not np.array_equal(want, yh[k * n_out * ch:(k + 1) * n_out * ch]):
            bad["resample"].append(k)
        img, _ = oracle_port.encode(want, ch, bps, rout, **FLAC8)
        fr = fres[k]
        if img != fh[fr.out_offset:fr.out_offset + fr.bytes].tobytes():
            bad["flac"].append(k)

    dt = _parallel(n_tracks, threads, one)
    out = {"verified_alac_port_decode": not bad["alac"],
           "verified_resample_vs_oracle": not bad["resample"],
           "verified_flac_vs_port": not bad["flac"],
           "verified_tracks": n_tracks - len(set(sum(bad.values(), []))),
           "verify_seconds": round(dt, 1)}
    # CPU baseline: reference binaries where they exist
    ref_ok = (os.path.exists(oracle_port.REF_ALACDEC) and os.path.exists(oracle_port.REF_FLACENC)
              and not args.no_cpu_baseline)
    nb = min(n_tracks, max(1, threads))
    fargs = [oracle_port.REF_FLACENC, "-c", str(ch), "-r", str(rout), "-b", str(bps), "-B",
             "4096", "-l", "12", "-P", "0", "-R", "6", "-m", "-e"]
    imgs = []
    if ref_ok:
        for k in range(nb):
            r = ares[k]
            mdat = alac_h[r.out_offset:r.out_offset + r.bytes].tobytes()
            sizes = [int(v) for v in fsb[r.first_frameset:r.first_frameset + r.n_framesets]]
            imgs.append(m4a.m4a_file(ch, bps, rin, 4096, n_in, mdat, sizes, create_date=1))
    same = []

    def base(k):
        if ref_ok:
            with tempfile.TemporaryDirectory() as d:
                fa = os.path.join(d, "a.m4a")
                with open(fa, "wb") as f:
                    f.write(imgs[k])
                p = subprocess.run([oracle_port.REF_ALACDEC, fa], capture_output=True, check=True)
                x = np.frombuffer(p.stdout, dtype=np.uint8).reshape(-1, 3)
                x = (x[:, 0].astype(np.int32) | (x[:, 1].astype(np.int32) << 8) |
                     (x[:, 2].astype(np.int8).astype(np.int32) << 16))
                rs = oracle_port.resample(x, ch, bps, rout / rin)
                raw = oracle_port.pcm_bytes(rs, bps)
                fo = os.path.join(d, "o.flac")
                subprocess.run(fargs + [fo], input=raw, stdout=subprocess.DEVNULL, check=True)
                with open(fo, "rb") as f:
                    img = f.read()
        else:
            x = sh[k * n_in * ch:(k + 1) * n_in * ch]
            rs = oracle_port.resample(x, ch, bps, rout / rin)
            img, _ = oracle_port.encode(rs, ch, bps, rout, **FLAC8)
        fr = fres[k]
        same.append(img == fh[fr.out_offset:fr.out_offset + fr.bytes].tobytes())

    bdt = _parallel(nb, threads, base)
    out["cpu_baseline"] = {
        "value": round(nb * n_out / bdt, 1), "unit": "frames/s", "cores": threads,
        "kind": "reference" if ref_ok else "port",
        "sample": "%d tracks x %d s, one track per worker, %d workers, %.1f s: %s"
                  % (nb, args.chain_seconds, threads, bdt,
                     "reference alacdec + flacenc processes (built from the reference's "
                     "src/decoders/alac.c, src/encoders/flac.c) around the resample port "
                     "(the reference's BEST-table resampler is unbuildable)" if ref_ok else
                     ("CPU restatements (--no-cpu-baseline: reference processes skipped)"
                      if args.no_cpu_baseline else "CPU restatements (oracle/_ref absent)")),
        "gpu_images_identical": all(same)}
    del yh, sh, fh, alac_h
    return out


def _device_equal(torch, eng, d_ptr, ref, n_tracks=1):
    """compare int32 at device address d_ptr with the tensor ref (on its
    device), copying through the engine (the process's one HIP runtime)
    -> (equal, first mismatching track or -1)"""
    got = torch.empty_like(ref)
    eng.copy_device(got.data_ptr(), d_ptr, ref.numel() * 4)
    if torch.equal(got, ref):
        return True, -1
    per = ref.numel() // max(1, n_tracks)
    for t in range(n_tracks):
        if not torch.equal(got[t * per:(t + 1) * per], ref[t * per:(t + 1) * per]):
            return False, t
    return False, n_tracks


def t2t_leg(args):
    """track2track in its true shape (reference
    audiotools/__init__.py:5494-5521, track2track:650-669): a driver process
    that imported audiotools but never touched the GPU forks one conversion
    process per WAV file, --t2t-procs at a time, each calling
    encode_flac(WaveReader) once and exiting -- fork, HIP-side setup and the
    encode all inside the clock.  The first conversion starts the encoder
    service (atgpu-encoderd), which then encodes every process's segments,
    batching concurrent ones.  The reference encoder runs the same files one
    process per file at the same count; every file is compared with it
    (tools/t2t_cold.py --fork, run as a child of this process)."""
    procs = max(1, args.t2t_procs)
    n_files = max(procs, args.t2t_files)
    cmd = [sys.executable, os.path.join(ROOT, "tools", "t2t_cold.py"), str(procs), str(n_files),
           "--fork", "--warm"]
    env = dict(os.environ)
    env.pop("ATG_ENCODER_SERVICE", None)
    # a socket name of this run's own: never an idle service of another run
    env["ATG_ENCODER_SOCKET"] = "atgpu-bench-%d" % os.getpid()
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    if p.returncode:
        return {"error": p.stderr[-2000:]}
    r = json.loads(p.stdout.strip().splitlines()[-1])
    out = {"metric": "track2track FLAC-8 encode, one forked process per file (%d at a time), "
                     "frames/s" % procs,
           "value": r["frames_per_s"], "unit": "frames/s", "processes": procs,
           "files": r["files"], "frames_per_file": r["frames_per_file"], "wall_s": r["wall_s"],
           "encoder": r["encoder"], "per_process_ms_mean": r["per_process_ms_mean"],
           "per_process_ms_max": r["per_process_ms_max"]}
    if r.get("warm"):
        # `value` includes the first conversion starting the service; the
        # same files again with the service up, as a session's later
        # conversions see it
        out["value_service_warm"] = r["warm"]["frames_per_s"]
        out["warm"] = r["warm"]
    ref = r.get("reference")
    if ref:
        out["cpu_baseline"] = {"value": ref["frames_per_s"], "unit": "frames/s",
                               "cores": procs, "kind": "reference",
                               "sample": "the same %d files, reference encoder "
                                         "(oracle/_ref/flacenc) one process per file, %d at a "
                                         "time, %.2f s" % (r["files"], procs, ref["wall_s"])}
        out["gpu_files_identical_to_reference"] = ref["files_identical"]
    return out


def rg_fallbacks():
    """tracks the last ReplayGain call could not certify and analysed again
    serially (replaygain.hip)"""
    import ctypes
    from audiotools import _atgpu
    lib = _atgpu.load_library()
    lib.atg_replaygain_fallback_tracks.restype = ctypes.c_uint32
    return int(lib.atg_replaygain_fallback_tracks())


def rg4_leg(args, torch, dist, world, rank, device, barrier, threads=16):
    """BASELINE config 4: ReplayGain album scan, 1024 tracks of
    --rg4-seconds s per GPU, one album per GPU: each
    rank's tracks are its album (title gains + the album gain/peak from the
    summed histogram); the albums' (gain, peak) go to every rank over RCCL
    (all_gather), and the whole set's gain/peak over an all-reduce of the
    histograms (SUM) and peaks (MAX).  Every track's title gain and peak,
    and the album gain and peak, are checked against the CPU oracle."""
    from audiotools import _atgpu
    n_tracks, n = 1024, args.rg4_seconds * 44100
    g = torch.Generator(device=device)
    g.manual_seed(77 + rank)
    t = torch.arange(n, device=device, dtype=torch.float32)
    x = torch.empty((n_tracks, n, 2), dtype=torch.int32, device=device)
    for k in range(0, n_tracks, 64):
        f = 90.0 + 13.0 * torch.arange(k, k + 64, device=device, dtype=torch.float32)
        amp = 2000.0 + 300.0 * (torch.arange(k, k + 64, device=device) % 50).float()
        tone = torch.sin(2 * np.pi * t[None, :] * f[:, None] / 44100.0) * amp[:, None]
        nz = torch.randint(-800, 800, (64, n, 2), device=device, generator=g, dtype=torch.int32)
        x[k:k + 64] = (tone[:, :, None].round().to(torch.int32) + nz).clamp(-32768, 32767)
    del t
    x = x.reshape(-1)
    torch.cuda.synchronize()
    tracks = [_atgpu.RgTrack(k * n, n, 2, 16, 44100, 0) for k in range(n_tracks)]
    hist = torch.zeros(12000, dtype=torch.int32, device=device)

    def step():
        res, peaks = _atgpu.replaygain_device(x.data_ptr(), tracks, 1, hist.data_ptr())
        gain = _atgpu.replaygain_hist_gain(hist.data_ptr(), 1)[0]
        return res, gain, peaks[0]

    steps = max(1, min(args.steps, 3))
    step()
    barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        res, album_gain, album_peak = step()
    barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        elapsed = reduce_max(torch, dist, elapsed, device)
        mine = torch.tensor([album_gain, album_peak], dtype=torch.float64, device=device)
        albums = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(albums, mine)
        albums = [tuple(float(v) for v in a.tolist()) for a in albums]
        pk = torch.tensor([album_peak], dtype=torch.float64, device=device)
        album_reduce(dist, world, hist, pk)
        set_gain = _atgpu.replaygain_hist_gain(hist.data_ptr(), 1)[0]
        set_peak = float(pk.item())
    else:
        albums = [(album_gain, album_peak)]
        set_gain, set_peak = album_gain, album_peak
    frames = n_tracks * n * world * steps / BLOCK
    out = {"metric": "ReplayGain album scan (config 4), FLAC-frame-equivalents/s",
           "value": round(frames / elapsed, 1), "unit": "frames/s",
           "ms_per_step": round(elapsed / steps * 1e3, 3), "steps": steps,
           "config": {"tracks_per_gpu": n_tracks, "seconds_per_track": args.rg4_seconds,
                      "album": "one per GPU"},
           "albums": [{"gain_db": a, "peak": p} for a, p in albums],
           "fallback_tracks_last_step": rg_fallbacks(),
           "all_albums": {"gain_db": set_gain, "peak": set_peak,
                          "collective": "all_gather (gain, peak) + all_reduce SUM uint32[12000]"
                                        " / MAX f64 (RCCL)" if world > 1 else "none (1 rank)"}}
    if rank == 0 and not args.no_verify:
        # every track's title gain and peak, and the album gain from the
        # summed oracle histograms, against the CPU oracle
        import oracle_port
        oracle_port.load()
        xh = x.cpu().numpy()
        bad, hists, peaks = [], [None] * n_tracks, [0.0] * n_tracks

        def one(k):
            A, pk = oracle_port.rg_title(xh[k * n * 2:(k + 1) * n * 2], 2, 16, 44100)
            hists[k], peaks[k] = A, pk
            if not (oracle_port.rg_gain(A) == res[k].title_gain and pk == res[k].title_peak):
                bad.append(k)

        vdt = _parallel(n_tracks, threads, one)
        want_album = oracle_port.rg_gain(np.sum(hists, axis=0).astype(np.uint32))
        album_ok = want_album == album_gain and max(peaks) == album_peak
        out["verified_tracks"] = n_tracks - len(bad)
        out["verified_album"] = album_ok
        out["verified_vs_oracle"] = not bad and album_ok
        out["verify_s"] = round(vdt, 1)
        out["cpu_baseline"] = {"value": round(n_tracks * n / BLOCK / vdt, 1),
                               "unit": "frames/s", "cores": threads, "kind": "port",
                               "sample": "the album's %d titles through oracle/replaygain_port.c"
                                         ", %d threads, %.1f s" % (n_tracks, threads, vdt)}
        # the drop-in: audiotools.calculate_replay_gain over the same album
        # (the callers' path under track2track --replay-gain: every title
        # read with read(4096), one GPU batch per device, the album from the
        # summed histogram), checked title by title against the oracle
        import audiotools
        mem = [_MemTrack(xh[k * n * 2:(k + 1) * n * 2], 2, 16, 44100) for k in range(n_tracks)]
        t1 = time.perf_counter()
        got = list(audiotools.calculate_replay_gain(mem))
        ddt = time.perf_counter() - t1
        dbad = [k for k, g in enumerate(got)
                if not (g[1] == oracle_port.rg_gain(hists[k]) and g[2] == peaks[k])]
        out["dropin_calculate_replay_gain"] = {
            "metric": "audiotools.calculate_replay_gain over the config-4 album, "
                      "FLAC-frame-equivalents/s (host PCM in, reader to gains)",
            "value": round(n_tracks * n / BLOCK / ddt, 1), "unit": "frames/s",
            "seconds": round(ddt, 3), "tracks": n_tracks,
            "verified_tracks": n_tracks - len(dbad),
            "verified_album": bool(got) and got[0][3] == want_album and
            got[0][4] == max(peaks),
            "gpu_calls": "one replaygain batch per device (replaygain.album_scan)"}
        del xh, hists
    del x, hist
    return out



def album_reduce(dist, world, hist, peak):
    """an album spread over ranks: SUM of the uint32 window histograms (held
    as int32; two's-complement sums are the same bits) and MAX of the peak,
    in place over RCCL -- the product's replaygain.album_allreduce (SURVEY
    8(e) ReplayGain row)"""
    if world > 1:
        from audiotools import replaygain
        replaygain.album_allreduce(hist, peak)


class _MemReader(object):
    """a PCMReader over int32 samples in host memory (bench stand-in for a
    decoded file: the drop-in leg times the GPU path, not disk reads)"""

    def __init__(self, samples, channels, bits, rate):
        self.samples, self.channels, self.bits_per_sample = samples, channels, bits
        self.sample_rate, self.channel_mask, self.pos = rate, 0x3 if channels == 2 else 0x4, 0

    def read(self, frames):
        from audiotools import pcm as _pcm
        a = self.samples[self.pos:self.pos + frames * self.channels]
        self.pos += len(a)
        return _pcm.FrameList._wrap(a, self.channels, self.bits_per_sample)

    def close(self):
        pass


class _MemTrack(object):
    """the AudioFile methods calculate_replay_gain calls, over _MemReader"""

    def __init__(self, samples, channels, bits, rate):
        self.s, self.ch, self.bits, self.rate = samples, channels, bits, rate

    def sample_rate(self):
        return self.rate

    def channels(self):
        return self.ch

    def total_frames(self):
        return len(self.s) // self.ch

    def to_pcm(self):
        return _MemReader(self.s, self.ch, self.bits, self.rate)




def replaygain_leg(args, torch, dist, world, rank, device, pcm, n_tracks, barrier):
    """ReplayGain title analysis of every track of the batch (replaygain.hip,
    SURVEY 8(a) G1-G5) plus one album over ALL ranks' tracks: each rank sums
    its tracks' window histograms on the GPU, then the 12000-bin uint32
    histogram is all-reduced (SUM, exact) and the album peak (MAX) over RCCL
    -- the one real exchange step of the path.  Returns the
    JSON object and per-track results for the CPU check."""
    from audiotools import _atgpu
    x = pcm.to(torch.int32)
    torch.cuda.synchronize()  # the library's streams read x
    n_samples = args.frames * BLOCK
    tracks = [_atgpu.RgTrack(t * n_samples, n_samples, 2, 16, 44100, 0)
              for t in range(n_tracks)]
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
    del x
    frames = n_tracks * args.frames * args.steps
    if world > 1:
        frames = reduce_sum(torch, dist, frames, device)
    fallbacks = rg_fallbacks()
    out = {"metric": "ReplayGain title analysis, FLAC-frame-equivalents/s (4096 PCM frames)",
           "value": round(frames / elapsed, 1), "unit": "frames/s",
           "ms_per_step": round(elapsed / args.steps * 1e3, 3),
           "fallback_tracks_last_step": fallbacks,
           "album": {"tracks": int(reduce_sum(torch, dist, n_tracks, device))
                     if world > 1 else n_tracks, "gain_db": album_gain,
                     "peak": album_peak,
                     "collective": "all_reduce SUM uint32[12000] + MAX f64 (RCCL)"
                                   if world > 1 else "none (1 rank)"},
           "bound": "serial fp64 IIR chain per track-channel (lane per track-channel)"}
    return out, res


def verify_replaygain(rg, rg_res, pcm_host, n_tracks, n_samples, threads):
    """every track's title gain and peak vs the CPU oracle (exact)"""
    import oracle_port
    oracle_port.load()
    bad = []

    def one(t):
        A, pk = oracle_port.rg_title(pcm_host[t * n_samples * 2:(t + 1) * n_samples * 2]
                                     .astype(np.int32), 2, 16, 44100)
        if not (oracle_port.rg_gain(A) == rg_res[t].title_gain and pk == rg_res[t].title_peak):
            bad.append(t)

    dt = _parallel(n_tracks, threads, one)
    rg["verified_vs_oracle"] = not bad
    rg["verified_tracks"] = n_tracks - len(bad)
    rg["cpu_baseline"] = {"value": round(n_tracks * (n_samples // BLOCK) / dt, 2),
                          "unit": "frames/s", "cores": threads, "kind": "port",
                          "sample": "oracle title analysis of all %d tracks, %d threads, %.1f s"
                                    % (n_tracks, threads, dt)}


def selftest(args):
    """the multi-rank harness on CPU (gloo): sharding, barrier + max-over-
    ranks clock, whole-job frame count, rank-0 JSON line.  The "step" is the
    CPU oracle encoding this rank's small tracks -- a harness check, not a
    measurement (metric says so)."""
    import torch
    import torch.distributed as dist
    import oracle_port
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")
    dev = torch.device("cpu")
    ids = shard(world, rank, args.tracks, args.scaling)
    rng = np.random.RandomState(7)
    pcms = {t: rng.randint(-3000, 3000, 2 * BLOCK * args.frames).astype(np.int32) for t in ids}
    for _ in range(args.warmup):
        for t in ids:
            oracle_port.encode(pcms[t], 2, 16, 44100, **FLAC8)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        for t in ids:
            oracle_port.encode(pcms[t], 2, 16, 44100, **FLAC8)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    frames = len(ids) * args.frames * args.steps
    if world > 1:
        elapsed = reduce_max(torch, dist, elapsed, dev)
        frames = reduce_sum(torch, dist, frames, dev)
    if rank == 0:
        print(json.dumps({"metric": "bench harness self-test (CPU oracle step; not a measurement)",
                          "value": round(frames / elapsed, 2), "unit": "frames/s",
                          "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "scaling": args.scaling, "selftest": True,
                          "tracks_total": int(frames // (args.frames * args.steps)),
                          "parallelism": "dp%d" % world}), flush=True)
    if world > 1:
        dist.destroy_process_group()


ALONE_LAUNCHES = 8
# the committed rocprofv3 kernel-stats pass of `bench.py --k2-profile` (every
# search launch a 1024-track batch alone on the device): the headline
# roofline's launch time is checked against its average
K2_PROFILE = "r06_k2_alone_kernel_stats.csv"
K2_KERNEL = "k_frame_search_ms"


def k2_alone(eng, opts, pcm, table, out_buf, out_cap, n):
    """mean search-kernel time (HIP events on the engine's main stream
    around the launch) over n batches encoded one at a time: the kernel's
    own duration, nothing queued beside or before it"""
    from audiotools import _atgpu
    ms = []
    for k in range(n + 1):
        eng.wait(eng.encode_device_async(opts, pcm.data_ptr(), _atgpu.PCM_S16, table, 2, 16,
                                         44100, out_buf.data_ptr(), out_cap))
        if k:
            ms.append(eng.kernel_times().get("subframe_search", 0.0))
    return sum(ms) / len(ms)


def k2_profile_avg():
    """(average ms, launches) of the search kernel in the committed
    rocprofv3 --kernel-trace --stats summary of `bench.py --k2-profile`"""
    import csv
    fn = os.path.join(ROOT, "profiles", K2_PROFILE)
    if not os.path.exists(fn):
        return None
    with open(fn) as f:
        for row in csv.DictReader(f):
            if K2_KERNEL in row.get("Name", ""):
                return float(row["AverageNs"]) / 1e6, int(row["Calls"])
    return None


def k2_profile_main(args):
    """--k2-profile: only the headline batch's search kernel, every launch
    one batch alone (what rocprofv3 --kernel-trace --stats summarises into
    profiles/r06_k2_alone_kernel_stats.csv)"""
    import torch
    from audiotools import _atgpu
    device = torch.device("cuda", 0)
    eng = _atgpu.Engine(0)
    opts = _atgpu.make_options(**FLAC8)
    n_samples = args.frames * BLOCK
    ids = list(range(args.tracks))
    pcm = synth_batch(torch, ids, n_samples, device)
    tracks = [(i * n_samples, n_samples) for i in range(len(ids))]
    _, out_cap = eng.bounds(opts, tracks, 2, 16)
    table = _atgpu.TrackTable(tracks)
    out = torch.empty(out_cap, dtype=torch.uint8, device=device)
    torch.cuda.synchronize()
    ms = k2_alone(eng, opts, pcm, table, out, out_cap, args.steps)
    print(json.dumps({"k2_profile": True, "launches": args.steps + 1,
                      "event_ms_mean": round(ms, 4), "tracks": len(ids),
                      "frames_per_track": args.frames}), flush=True)
    eng.close()
    return 0


def narrow_leg(args, torch, dist, world, device, eng, opts, pcm, tracks, out_full, res_full,
               barrier):
    """frames/s of narrow batches (the first n tracks of the config-2 batch)
    at each in-flight depth -- "auto" = the engine's own choice
    (atg_engine_set_inflight(0), engine.hip auto_depth), the caller keeping
    eng.inflight() batches in flight; every image of the last batch
    byte-compared with the full batch's image of the same track"""
    from audiotools import _atgpu
    widths = [int(x) for x in args.narrow.split(",") if x.strip()]
    depths = [x.strip() for x in args.narrow_depths.split(",") if x.strip()]
    out = {}
    for n in widths:
        n = min(n, len(tracks))
        sub = tracks[:n]
        _, cap = eng.bounds(opts, sub, 2, 16)
        table = _atgpu.TrackTable(sub)
        per = {}
        for spec in depths:
            eng.set_inflight(0 if spec == "auto" else int(spec))
            bufs = []
            pend = []

            def run(steps):
                last, d = None, None
                for k in range(steps):
                    if d is not None and len(bufs) < d:
                        bufs.append(torch.empty(cap, dtype=torch.uint8, device=device))
                    elif d is None and not bufs:
                        bufs.append(torch.empty(cap, dtype=torch.uint8, device=device))
                    pend.append((k, eng.encode_device_async(
                        opts, pcm.data_ptr(), _atgpu.PCM_S16, table, 2, 16, 44100,
                        bufs[k % len(bufs)].data_ptr(), cap)))
                    d = eng.inflight()  # the automatic depth is set by the first enqueue
                    if len(pend) >= d:
                        last = (pend[0][0], eng.wait(pend.pop(0)[1]))
                while pend:
                    last = (pend[0][0], eng.wait(pend.pop(0)[1]))
                return last, d

            run(34)  # warm-up: fills the buffer ring at any depth
            barrier()
            t0 = time.perf_counter()
            (k_last, r), d = run(args.steps)
            barrier()
            dt = time.perf_counter() - t0
            if world > 1:
                dt = reduce_max(torch, dist, dt, device)
            kt = eng.kernel_times()
            last = bufs[k_last % len(bufs)]
            bad = 0
            for t in range(n):
                a = last[r[t].out_offset:r[t].out_offset + r[t].bytes]
                b = out_full[res_full[t].out_offset:res_full[t].out_offset + res_full[t].bytes]
                if r[t].bytes != res_full[t].bytes or not torch.equal(a, b):
                    bad += 1
            key = "inflight_auto" if spec == "auto" else "inflight_%s" % spec
            per[key] = {
                "value": round(n * args.frames * args.steps / dt, 1), "unit": "frames/s",
                "ms_per_step": round(dt / args.steps * 1e3, 3), "inflight": d,
                "kernel_ms": {k: round(v, 3) for k, v in kt.items()},
                "verified_tracks": n - bad, "mismatches": bad}
            del bufs
        eng.set_inflight(max(3, args.inflight))
        out[str(n)] = per
    return {"tracks_per_batch": out,
            "note": "the first n tracks of the config-2 batch per step, pipelined; "
                    "inflight_auto = the engine's default (automatic) depth; "
                    "images compared with the full batch's (the same tracks' bytes)"}


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    args = parse_args(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # spawn the ranks before anything initialises a GPU (never re-exec)
        return launch(args, argv)
    if args.selftest:
        return selftest(args)
    if args.k2_profile:
        return k2_profile_main(args)
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
    ids = shard(world, rank, args.tracks, args.scaling)
    n_tracks = len(ids)
    pcm = synth_batch(torch, ids, n_samples, device)
    tracks = [(i * n_samples, n_samples) for i in range(n_tracks)]
    n_frames, out_cap = eng.bounds(opts, tracks, 2, 16)
    table = _atgpu.TrackTable(tracks)
    # `depth` output buffers: batch k is waited once batch k + depth - 1 is
    # enqueued (atg_flac_encode_device_async), so batch k's MD5 chains and
    # headers run under the next batches' search chains; every batch is
    # complete inside the clock.  Depth 12 (rolled MD5: each batch's chains
    # advance a slice per later enqueue) measured 7.99 ms per step against
    # 8.30 at 3, 8.07-8.11 at 8 and 8.06 at 16 (profiles/r05_zs_inflight.json)
    depth = args.inflight
    if depth > 3:
        eng.set_inflight(depth)
    outs = [torch.empty(out_cap, dtype=torch.uint8, device=device) for _ in range(depth)]
    torch.cuda.synchronize()
    pending = []

    def step(k):
        t = eng.encode_device_async(opts, pcm.data_ptr(), _atgpu.PCM_S16, table, 2, 16, 44100,
                                    outs[k % depth].data_ptr(), out_cap)
        pending.append(t)
        return eng.wait(pending.pop(0)) if len(pending) >= depth else None

    def drain():
        r = None
        while pending:
            r = eng.wait(pending.pop(0))
        return r

    for k in range(args.warmup):
        step(k)
    if args.warmup:
        drain()

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    kt_sum = {}
    barrier()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(k)
        if k:
            for name, v in eng.kernel_times().items():
                kt_sum[name] = kt_sum.get(name, 0.0) + v
    res = drain()
    for name, v in eng.kernel_times().items():
        kt_sum[name] = kt_sum.get(name, 0.0) + v
    barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        elapsed = reduce_max(torch, dist, elapsed, device)
    out = outs[(args.steps - 1) % depth]
    # the batches below write their own buffers: `out` holds the images the
    # parity check and the decode leg read
    outs = [torch.empty(out_cap, dtype=torch.uint8, device=device) for _ in range(depth)]

    def timed(tbl, steps):
        """wall time of `steps` pipelined batches of table `tbl` (a
        TrackTable, or a callable k -> TrackTable), max over ranks"""
        barrier()
        t1 = time.perf_counter()
        for k in range(steps):
            tb = tbl(k) if callable(tbl) else tbl
            t = eng.encode_device_async(opts, pcm.data_ptr(), _atgpu.PCM_S16, tb, 2, 16, 44100,
                                        outs[k % depth].data_ptr(), out_cap)
            pending.append(t)
            if len(pending) >= depth:
                eng.wait(pending.pop(0))
        drain()
        barrier()
        dt = time.perf_counter() - t1
        return reduce_max(torch, dist, dt, device) if world > 1 else dt

    # ---- strong scaling: the 1024-track batch split over the
    # ranks, timed in the same run as the weak line above
    strong = None
    if world > 1 and args.scaling == "weak":
        n_s = len(shard(world, rank, args.tracks, "strong"))
        st_table = _atgpu.TrackTable(tracks[:n_s])
        # a narrow rank batch keeps more batches in flight so the per-track
        # MD5 chains (~12.5 ms per 1 MiB track whatever the width) stay off
        # the step: the engine's automatic depth (engine.hip auto_depth,
        # rolled MD5), read after the first enqueue
        _, s_cap = eng.bounds(opts, tracks[:n_s], 2, 16)
        s_outs = [torch.empty(s_cap, dtype=torch.uint8, device=device) for _ in range(32)]
        eng.set_inflight(0)
        s_depth = 0

        def s_timed(steps):
            nonlocal s_depth
            barrier()
            t1 = time.perf_counter()
            pend = []
            for k in range(steps):
                pend.append(eng.encode_device_async(opts, pcm.data_ptr(), _atgpu.PCM_S16,
                                                    st_table, 2, 16, 44100,
                                                    s_outs[k % 32].data_ptr(), s_cap))
                s_depth = eng.inflight()
                if len(pend) >= s_depth:
                    eng.wait(pend.pop(0))
            while pend:
                eng.wait(pend.pop(0))
            barrier()
            dt = time.perf_counter() - t1
            return reduce_max(torch, dist, dt, device)

        s_timed(34)
        dt = s_timed(args.steps)
        eng.set_inflight(max(3, args.inflight))
        del s_outs
        tot = reduce_sum(torch, dist, n_s * args.frames * args.steps, device)
        strong = {"value": round(tot / dt, 1), "unit": "frames/s",
                  "ms_per_step": round(dt / args.steps * 1e3, 3),
                  "tracks_total": args.tracks, "tracks_per_gpu": n_s, "inflight": s_depth,
                  "bound": "per-track MD5 chain (~12.5 ms per 1 MiB track, serial): a narrow "
                           "rank keeps %d batches in flight, their chains advanced together "
                           "(rolled MD5)" % s_depth}
    # ---- narrow batches (SURVEY 8(e) strong scaling: a rank's share of the
    # 1024-track job), one GPU, pipelined at several in-flight depths; the
    # last batch's images are compared with the full batch's (the same
    # tracks' PCM, so the same bytes: the full batch is checked against the
    # port below)
    narrow = narrow_leg(args, torch, dist, world, device, eng, opts, pcm, tracks, out, res,
                        barrier) if args.narrow else None
    # ---- the search kernel with one batch in flight: in the pipelined loop
    # above the batches behind run their LPC kernels (slot stream) beside it
    sub_alone_ms = k2_alone(eng, opts, pcm, table, outs[0], out_cap, ALONE_LAUNCHES)
    # ---- per-batch host planning: every step a new track geometry (the
    # plan cache misses; engine.hip get_plan), against the fixed geometry
    plan_steps = min(args.steps, 10)

    def varied(k):
        lens = [n_samples - 4096 * ((i + k) % 3) for i in range(n_tracks)]
        return _atgpu.TrackTable([(i * n_samples, lens[i]) for i in range(n_tracks)])

    tables = [varied(k) for k in range(plan_steps)]  # built outside the clock
    dt_var = timed(lambda k: tables[k], plan_steps)
    dt_fix = timed(table, plan_steps)
    plan_miss = {"steps": plan_steps,
                 "ms_per_step_new_geometry": round(dt_var / plan_steps * 1e3, 3),
                 "ms_per_step_same_geometry": round(dt_fix / plan_steps * 1e3, 3),
                 "host_plan_ms_per_batch": round((dt_var - dt_fix) / plan_steps * 1e3, 3),
                 "note": "each step's batch has different track lengths (frames drop per "
                         "track by 0-2 frames in turn): the host plan, frame/track tables "
                         "and their upload are redone every step"}
    del tables
    del outs
    kt = {k: v / args.steps for k, v in kt_sum.items()}
    out_bytes = sum(int(r.bytes) for r in res)
    frame_bytes = out_bytes - HEADER_BYTES * len(res)
    total_frames = n_frames * args.steps
    if world > 1:
        total_frames = reduce_sum(torch, dist, total_frames, device)

    share, share_info = cpu_share()
    threads = args.cpu_threads or share
    pcm_host = pcm.cpu().numpy()
    host_out = out.cpu().numpy()
    images = [host_out[r.out_offset:r.out_offset + r.bytes].tobytes() for r in res]
    del host_out

    # ---- parity: every image of the batch vs the CPU port (outside the
    # timed region); the port's timing is the N-thread port baseline
    verified = None
    port = None
    if not args.no_verify:
        want, port_dt = port_encode_all(pcm_host, n_tracks, n_samples, threads)
        bad = [t for t in range(n_tracks) if want[t] != images[t]]
        verified = {"vs": "CPU port oracle/flac_port.c (pinned to the reference encoder)",
                    "tracks": n_tracks, "mismatches": len(bad), "ok": not bad}
        port = {"value": round(n_tracks * args.frames / port_dt, 2), "unit": "frames/s",
                "cores": threads, "kind": "port",
                "sample": "all %d tracks x %d frames, %d threads, %.1f s"
                          % (n_tracks, args.frames, threads, port_dt)}
        del want

    decode = convert = rg = rg_res = resample = host = None
    # the legs below keep the engine's default rotation (three slots, each
    # with its aux stream from creation: deeper rotations add streams)
    eng.set_inflight(3)
    if not args.no_host:
        host = host_leg(args, torch, dist, world, device, eng, opts, pcm_host, tracks, n_frames,
                        images, barrier)
    if not args.no_decode:
        decode = decode_leg(args, torch, dist, world, device, eng, out, res, pcm, pcm_host,
                            n_frames, barrier)
        if rank == 0:
            convert = convert_leg(args, torch, device, pcm)
        resample = resample_leg(args, torch, dist, world, device, pcm, n_tracks, barrier,
                                threads, rank == 0 and not args.no_verify)
        rg, rg_res = replaygain_leg(args, torch, dist, world, rank, device, pcm, n_tracks,
                                    barrier)
    t2t = rg4 = None
    if not args.no_t2t and rank == 0 and world == 1:
        t2t = t2t_leg(args)
    if not args.no_rg4:
        rg4 = rg4_leg(args, torch, dist, world, rank, device, barrier, threads)
    chain = None
    if not args.no_chain:
        chain = chain_leg(args, torch, dist, world, device, barrier, threads,
                          rank == 0 and not args.no_verify)

    if rank != 0:
        eng.close()
        _atgpu.close_all()
        if world > 1:
            dist.destroy_process_group()
        return 0

    value = total_frames / elapsed
    # ---- rooflines.  Algorithmic bytes per launch:
    # every kernel that reads the batch reads its PCM once (16,384 B per
    # 4096-sample stereo frame); the packer also writes the compressed frames
    pcm_bytes = n_tracks * n_samples * 2 * 2
    alg = {"lpc_analyze": pcm_bytes, "subframe_search": pcm_bytes,
           "frame_pack": pcm_bytes + frame_bytes, "track_md5": pcm_bytes,
           "frame_decide": 0, "track_scan": 0, "stream_header": out_bytes - frame_bytes}
    main_k = {k: v for k, v in kt.items() if k in MAIN_STREAM}
    dom = max(main_k, key=main_k.get)
    dom_ms = main_k[dom]  # live event span in the pipelined loop
    alg_bytes = alg.get(dom, pcm_bytes)
    traffic = (load_profile_json("pmc_traffic.json") or {}).get(dom)
    # the roofline's kernel time is the search kernel's own duration (one
    # batch on the device, HIP events around the launch): the live span
    # above also holds the time the kernel's stream waits behind the batches
    # beside it, and can exceed the step
    ms_step = elapsed / args.steps * 1e3
    assert sub_alone_ms <= ms_step, (sub_alone_ms, ms_step)
    achieved = alg_bytes / (sub_alone_ms / 1e3) / 1e9
    prof = k2_profile_avg()
    roofline = {"bound": "hbm", "kernel": "subframe_search", "achieved": round(achieved, 2),
                "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                "alg_bytes_per_launch": alg_bytes, "launch_ms": round(sub_alone_ms, 4),
                "launch_ms_source": "HIP events around the search launch, %d batches encoded "
                                    "one at a time after the clock" % ALONE_LAUNCHES,
                "launch_ms_le_ms_per_step": True,
                "live_span_ms": round(dom_ms, 4),
                "live_span_note": "event span of the longest main-stream kernel (%s) in the "
                                  "pipelined loop: includes queueing behind the batches in "
                                  "flight, not a kernel duration, not used for frac" % dom,
                "profile": None}
    if prof:
        roofline["profile"] = {
            "file": "profiles/" + K2_PROFILE, "kernel": K2_KERNEL + "<short>",
            "avg_ms": round(prof[0], 4), "calls": prof[1],
            "frac": round(alg_bytes / (prof[0] / 1e3) / 1e9 / HBM_PEAK_GBS, 5),
            "launch_ms_vs_profile": round(sub_alone_ms / prof[0], 4)}
    # integer-VALU roofline of the subframe search: algorithmic
    # MACs = sum over the 4 candidate subframes of the 12 LPC orders
    # (1+..+12 = 78 taps x 4096 samples) + FIXED orders 1..4 (10 taps) --
    # 2 MACs per v_dot2 lane-op, 64 lanes per wave instruction
    sub_ms = sub_alone_ms  # the kernel's own duration, as the HBM roofline above
    macs_per_frame = 4 * (78 + 10) * BLOCK
    alg_wave_insts = n_frames * macs_per_frame / 2.0 / 64.0
    pmc = (load_profile_json("pmc_valu.json") or {}).get("subframe_search") or {}
    valu = {"kernel": "subframe_search", "bound": "valu", "unit": "wave-instructions/s",
            "peak": VALU_PEAK_WAVE_INSTS,
            "alg_mac_wave_insts_per_launch": alg_wave_insts,
            "alg_mac_frac": round(alg_wave_insts / (sub_ms / 1e3) / VALU_PEAK_WAVE_INSTS, 4)
            if sub_ms else None,
            "launch_ms": round(sub_ms, 4)}
    if pmc.get("SQ_INSTS_VALU") and sub_ms:
        # PMC instruction count per launch (profiles/pmc_valu.json, same
        # batch shape) over the live launch time
        per_launch = pmc["SQ_INSTS_VALU"] * (n_frames / pmc.get("frames", n_frames))
        valu["issued_wave_insts_per_launch"] = per_launch
        valu["issue_frac"] = round(per_launch / (sub_ms / 1e3) / VALU_PEAK_WAVE_INSTS, 4)
        valu["pmc_source"] = pmc.get("source")
    step_alg = pcm_bytes + out_bytes
    step_hbm = {"alg_bytes_per_step": step_alg,
                "achieved": round(step_alg / (elapsed / args.steps) / 1e9, 2),
                "frac": round(step_alg / (elapsed / args.steps) / 1e9 / HBM_PEAK_GBS, 5)}

    # ---- CPU baselines on this host's cores
    cpu = None
    if not args.no_cpu_baseline:
        import oracle_port
        nref = min(args.cpu_ref_tracks, n_tracks)
        ref = ref_encode_sample(pcm_host, nref, n_samples, threads)
        t1 = min(2, n_tracks)
        _, dt1 = port_encode_all(pcm_host, t1, n_samples, 1)
        port1 = {"value": round(t1 * args.frames / dt1, 2), "unit": "frames/s", "cores": 1,
                 "kind": "port", "sample": "%d tracks x %d frames, 1 thread, %.1f s"
                                           % (t1, args.frames, dt1)}
        if ref is not None:
            ref_images, rdt = ref
            ref_ok = all(ref_images[t] == images[t] for t in range(nref))
            # -j nproc as track2track would on this host: one process per
            # visible CPU; the cgroup quota (cpu_share) bounds what it gets
            nproc = os.cpu_count() or threads
            refn = ref_encode_sample(pcm_host, nref, n_samples, nproc) if nproc > threads \
                else None
            cpu = {"value": round(nref * args.frames / rdt, 2), "unit": "frames/s",
                   "cores": threads, "kind": "reference",
                   "sample": "reference encoder (oracle/_ref/flacenc, built from the "
                             "reference's src/encoders/flac.c) on %d of the batch's tracks x "
                             "%d frames, one process per track, %d at a time, %.1f s"
                             % (nref, args.frames, threads, rdt),
                   "gpu_images_identical": ref_ok}
            if refn is not None:
                cpu["nproc"] = {"value": round(nref * args.frames / refn[1], 2),
                                "unit": "frames/s", "processes": nproc,
                                "sample": "the same %d tracks, %d processes at a time "
                                          "(os.cpu_count()), %.1f s; the cgroup CPU quota "
                                          "%s CPUs bounds it" % (nref, nproc, refn[1],
                                                                 share_info.get(
                                                                     "cgroup_quota_cpus"))}
        else:
            cpu = dict(port) if port else dict(port1)
            cpu["note"] = "oracle/_ref absent: port timing"
        cpu["cpu_model"] = cpu_model()
        cpu["host_cpus"] = os.cpu_count()
        cpu["cpu_share"] = share_info
        cpu["port_1_thread"] = port1
        if port:
            cpu["port_n_threads"] = port
        cal = load_profile_json("r02_cpu_calibration.json")
        if cal:
            cpu["calibration"] = cal.get("summary")
        if rg is not None:
            verify_replaygain(rg, rg_res, pcm_host, n_tracks, n_samples, threads)

    line = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        # SURVEY 8(d)'s timer: pinned host PCM in, host images out, PCIe
        # transfers inside the clock (the host_to_host leg, same batch)
        "value_host_to_host": host.get("value") if isinstance(host, dict) else None,
        "higher_is_better": True,
        "scaling": args.scaling,
        "vs_baseline": None,
        "dtype": "int32 residuals / f64 LPC analysis (s16 PCM in)",
        "data": "synthetic (seeded sine+noise, 5% white noise, 2% silent tracks)",
        "config": {"workload": "FLAC-8 batch encode, %d tracks x %d frames x 4096 samples "
                               "per GPU, 44.1 kHz 16-bit stereo, PCM and .flac images in HBM"
                               % (n_tracks, args.frames),
                   "tracks_per_gpu": n_tracks, "frames_per_track": args.frames,
                   "block_size": 4096, "preset": "FLAC-8 (-l 12 -m -e -R 6)",
                   "parallelism": "dp%d (tracks sharded per GPU, %s scaling)"
                                  % (world, args.scaling)},
        "roofline": roofline,
        "roofline_valu": valu,
        "step_hbm": step_hbm,
        "kernel_ms": {k: round(v, 4) for k, v in kt.items()},
        "compressed_bytes_per_frame": round(frame_bytes / n_frames, 1),
        "verified_vs_oracle": verified,
        "cpu_baseline": cpu,
        "decode": decode,
        "convert": convert,
        "replaygain": rg,
        "host_to_host": host,
        "resample": resample,
        "chain": chain,
        "replaygain_config4": rg4,
        "track2track": t2t,
        "strong_scaling": strong if world > 1 else {"note": "1 GPU: the same batch as value"},
        "narrow_batches": narrow,
        "plan_per_batch": plan_miss,
    }
    print(json.dumps(line), flush=True)
    # every handle closed here, in order, not from interpreter teardown
    # 
    eng.close()
    _atgpu.close_all()
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
