"""track2track in its true shape: one fresh process per track.

track2track runs every conversion in a new multiprocessing.Process
(ExecProgressQueue.spawn, reference audiotools/__init__.py:5494-5521;
track2track:650-669), so under the drop-in each track pays interpreter
start, imports, HIP init, code-object load, engine creation and its first
launches before it encodes.  This probe runs N WAV files with at most J
processes alive, one process per file, from a parent that never touches the
GPU, and breaks the per-process time into phases; the reference encoder
(oracle/_ref/flacenc, one process per file, J at a time) runs the same files
beside it when present.

  python tools/t2t_cold.py J [N] [--frames F] [--fork] [--own-engine] [--warm]  -> JSON line
    --fork: the parent imports audiotools and forks a process per file
    (multiprocessing, as track2track); default: a fresh interpreter each
    --warm (with --fork): the same files converted a second time, timed
    apart, with the encoder service the first run started still up
    --own-engine: ATG_ENCODER_SERVICE=off (every process its own engine)
  python tools/t2t_cold.py --one in.wav out.flac   (a child)
"""
import time

T_START = time.time()  # noqa: E402  (first statement: process start, near enough)

import json  # noqa: E402
import os  # noqa: E402
import struct  # noqa: E402
import subprocess  # noqa: E402
import sys  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
FLAC8 = dict(block_size=4096, max_lpc_order=12, min_residual_partition_order=0,
             max_residual_partition_order=6, mid_side=1, adaptive_mid_side=0,
             exhaustive_model_search=1)


def hip_init():
    """with an engine per process (ATG_ENCODER_SERVICE=off) bring HIP up
    first to time it apart; with the encoder service the process never does"""
    if os.environ.get("ATG_ENCODER_SERVICE") == "off":
        import ctypes
        hip = ctypes.CDLL("libamdhip64.so")
        n = ctypes.c_int()
        hip.hipGetDeviceCount(ctypes.byref(n))
    return time.time()


def child(wav_in, flac_out):
    t = {"start": T_START}
    import numpy  # noqa: F401
    t["numpy"] = time.time()
    sys.path.insert(0, os.path.join(ROOT, "python-audio-tools_amd"))
    import audiotools
    from audiotools import encoders, wav
    t["audiotools"] = time.time()
    t["hip_init"] = hip_init()
    offs = encoders.encode_flac(flac_out, audiotools.BufferedPCMReader(wav.WaveReader(wav_in)),
                                **FLAC8)
    t["encode"] = time.time()
    print(json.dumps({"t": t, "frames": len(offs)}), flush=True)
    return 0


def fork_child(wav_in, flac_out, q, t_fork):
    """the body of a track2track conversion process (a forked
    multiprocessing.Process, ExecProgressQueue.spawn): audiotools is already
    imported by the parent, which never touched the GPU"""
    import audiotools
    from audiotools import encoders, wav
    t = {"start": time.time()}
    t["hip_init"] = hip_init()
    offs = encoders.encode_flac(flac_out, audiotools.BufferedPCMReader(wav.WaveReader(wav_in)),
                                **FLAC8)
    t["encode"] = time.time()
    q.put(json.dumps({"t": t, "frames": len(offs), "t_fork": t_fork}))


def run_forks(files, gdir, j):
    """one forked process per file, at most j alive (track2track -j);
    -> (wall s, [(fork time, child JSON)])"""
    import multiprocessing as mp
    ctx = mp.get_context("fork")
    q = ctx.Queue()
    t0 = time.time()
    pending, alive, done = list(files), [], []
    while pending or alive:
        while pending and len(alive) < j:
            fn = pending.pop(0)
            out = os.path.join(gdir, os.path.basename(fn)[:-4] + ".flac")
            ts = time.time()
            p = ctx.Process(target=fork_child, args=(fn, out, q, ts))
            p.start()
            alive.append((ts, p))
        still = []
        for ts, p in alive:
            if p.exitcode is None:
                still.append((ts, p))
            elif p.exitcode:
                raise RuntimeError("conversion process failed: %d" % p.exitcode)
            else:
                done.append(ts)
        alive = still
        time.sleep(0.0005)
    wall = time.time() - t0
    outs = [q.get() for _ in done]
    return wall, [(json.loads(o)["t_fork"], o) for o in outs]


def write_wavs(d, n_files, frames):
    import numpy as np
    rng = np.random.default_rng(7)
    files = []
    n = frames * 4096
    for k in range(n_files):
        x = np.cumsum(rng.integers(-300, 301, 2 * n)).clip(-30000, 30000).astype("<i2")
        data = x.tobytes()
        fn = os.path.join(d, "t%04d.wav" % k)
        with open(fn, "wb") as f:
            f.write(struct.pack("<4sI4s4sIHHIIHH4sI", b"RIFF", 36 + len(data), b"WAVE",
                                b"fmt ", 16, 1, 2, 44100, 44100 * 4, 4, 16, b"data",
                                len(data)))
            f.write(data)
        files.append(fn)
    return files


def _profiler_noise_only(err):
    """stderr holding nothing but a profiler's own log lines (rocprofv3
    preloads itself into every child of a profiled run)"""
    lines = [ln for ln in err.decode(errors="replace").splitlines() if ln.strip()]
    return all("rocprofv3" in ln or "rocprofiler" in ln for ln in lines)


def run_pool(cmds, j, tolerate_profiler=False):
    """run the commands, at most j alive; -> (wall s, [(spawn time, stdout)]).
    tolerate_profiler: a child that exits non-zero with only profiler log
    lines on stderr counts as done (the reference encoder's pipeline under
    rocprofv3; its output files are compared afterwards, so a real failure
    still shows as files_identical false)"""
    t0 = time.time()
    pending, alive, done = list(cmds), [], []
    while pending or alive:
        while pending and len(alive) < j:
            c = pending.pop(0)
            alive.append((time.time(), subprocess.Popen(c, stdout=subprocess.PIPE,
                                                        stderr=subprocess.PIPE)))
        still = []
        for ts, p in alive:
            if p.poll() is None:
                still.append((ts, p))
                continue
            out, err = p.communicate()
            if p.returncode and not (tolerate_profiler and _profiler_noise_only(err)):
                raise RuntimeError("child failed: %s" % err.decode()[-2000:])
            done.append((ts, out.decode()))
        alive = still
        time.sleep(0.0005)
    return time.time() - t0, done


def main():
    if sys.argv[1] == "--one":
        return child(sys.argv[2], sys.argv[3])
    import tempfile
    j = int(sys.argv[1])
    n_files = int(sys.argv[2]) if len(sys.argv) > 2 and not sys.argv[2].startswith("-") else 4 * j
    frames = 64
    if "--frames" in sys.argv:
        frames = int(sys.argv[sys.argv.index("--frames") + 1])
    with tempfile.TemporaryDirectory(dir="/dev/shm" if os.path.isdir("/dev/shm") else None) as d:
        files = write_wavs(d, n_files, frames)
        gdir = os.path.join(d, "gpu")
        os.mkdir(gdir)
        fork = "--fork" in sys.argv
        own = "--own-engine" in sys.argv
        if own:  # inherited by the children
            os.environ["ATG_ENCODER_SERVICE"] = "off"
        if fork:
            # the parent imports audiotools (never the GPU), as track2track's
            # process does before ExecProgressQueue forks the conversions
            sys.path.insert(0, os.path.join(ROOT, "python-audio-tools_amd"))
            import audiotools  # noqa: F401
            from audiotools import encoders  # noqa: F401
            wall, done = run_forks(files, gdir, j)
            keys = ["hip_init", "encode"]
            warm = None
            if "--warm" in sys.argv:
                # the same files again with the encoder service the first
                # run started still up (a session's later conversions)
                wdir = os.path.join(d, "gpu_warm")
                os.mkdir(wdir)
                wwall, _ = run_forks(files, wdir, j)
                same_w = all(open(os.path.join(wdir, os.path.basename(f)[:-4] + ".flac"),
                                  "rb").read() ==
                             open(os.path.join(gdir, os.path.basename(f)[:-4] + ".flac"),
                                  "rb").read() for f in files)
                warm = {"wall_s": round(wwall, 3),
                        "frames_per_s": round(n_files * frames / wwall, 1),
                        "files_identical_to_first_run": same_w}
        else:
            cmds = [[sys.executable, os.path.abspath(__file__), "--one", fn,
                     os.path.join(gdir, os.path.basename(fn)[:-4] + ".flac")] for fn in files]
            wall, done = run_pool(cmds, j)
            keys = ["numpy", "audiotools", "hip_init", "encode"]
            warm = None
        phases = {}
        for ts, out in done:
            t = json.loads(out.strip().splitlines()[-1])["t"]
            phases.setdefault("spawn_to_start", []).append(max(0.0, t["start"] - ts))
            prev = t["start"]
            for k in keys:
                phases.setdefault(k, []).append(t[k] - prev)
                prev = t[k]
        total_frames = n_files * frames
        res = {"mode": "fork" if fork else "spawn",
               "encoder": "engine per process" if own else "encoder service (atgpu-encoderd)",
               "processes": j, "files": n_files,
               "frames_per_file": frames,
               "wall_s": round(wall, 3), "frames_per_s": round(total_frames / wall, 1),
               "per_process_ms_mean": {k: round(1e3 * sum(v) / len(v), 1)
                                       for k, v in phases.items()},
               "per_process_ms_max": {k: round(1e3 * max(v), 1) for k, v in phases.items()}}
        if warm:
            res["warm"] = warm
        ref = os.path.join(ROOT, "oracle", "_ref", "flacenc")
        if os.path.exists(ref):
            rdir = os.path.join(d, "ref")
            os.mkdir(rdir)
            rc = [["sh", "-c", "tail -c +45 %s | %s -c 2 -r 44100 -b 16 -B 4096 -l 12 -P 0 "
                   "-R 6 -m -e %s > /dev/null" % (fn, ref, os.path.join(rdir, os.path.basename(
                       fn)[:-4] + ".flac"))] for fn in files]
            rwall, _ = run_pool(rc, j, tolerate_profiler=True)
            def _read(path):
                try:
                    with open(path, "rb") as fh:
                        return fh.read()
                except OSError:
                    return None
            same = all(_read(os.path.join(rdir, os.path.basename(f)[:-4] + ".flac")) is not None
                       and _read(os.path.join(gdir, os.path.basename(f)[:-4] + ".flac"))
                       == _read(os.path.join(rdir, os.path.basename(f)[:-4] + ".flac"))
                       for f in files)
            res["reference"] = {"wall_s": round(rwall, 3),
                                "frames_per_s": round(total_frames / rwall, 1),
                                "files_identical": same}
        print(json.dumps(res), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
