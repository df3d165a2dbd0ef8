"""track2track leg breakdown on the GPU box: N processes x encode_flac on
WAV files, each worker timing its engine.encode_frames calls apart from the
rest (WAV parsing, MD5, file I/O).  Usage: t2t_probe.py PROCS [TRACKS]"""
import json, os, struct, subprocess, sys, tempfile, time
import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "python-audio-tools_amd"))
FLAC8 = dict(block_size=4096, max_lpc_order=12, min_residual_partition_order=0,
             max_residual_partition_order=6, mid_side=1, adaptive_mid_side=0,
             exhaustive_model_search=1)


def worker(list_file, out_dir, go):
    import audiotools
    from audiotools import _atgpu, encoders, wav
    _atgpu.load_library()
    eng = _atgpu.engine()
    orig = eng.encode_frames
    acc = {"eng": 0.0, "calls": 0, "each_ms": []}

    def timed(*a, **k):
        t = time.perf_counter()
        r = orig(*a, **k)
        acc["eng"] += time.perf_counter() - t
        acc["each_ms"].append(round(1e3 * (time.perf_counter() - t), 2))
        acc["calls"] += 1
        return r
    eng.encode_frames = timed
    names = [ln.strip() for ln in open(list_file) if ln.strip()]
    print(json.dumps({"ready": True}), flush=True)
    while not os.path.exists(go):
        time.sleep(0.001)
    t0 = time.perf_counter()
    frames = 0
    for fn in names:
        out = os.path.join(out_dir, os.path.basename(fn)[:-4] + ".flac")
        frames += len(encoders.encode_flac(out, audiotools.BufferedPCMReader(wav.WaveReader(fn)),
                                           **FLAC8))
    print(json.dumps({"frames": frames, "seconds": time.perf_counter() - t0, **acc,
                      "kernel_ms": eng.kernel_times()}), flush=True)


def main():
    if sys.argv[1] == "--worker":
        return worker(*sys.argv[2:5])
    procs = int(sys.argv[1])
    tracks = int(sys.argv[2]) if len(sys.argv) > 2 else 8 * procs
    n = 64 * 4096
    rng = np.random.default_rng(7)
    with tempfile.TemporaryDirectory(dir="/dev/shm") as d:
        files = []
        for t in range(tracks):
            x = np.cumsum(rng.integers(-300, 301, 2 * n)).clip(-30000, 30000).astype("<i2")
            data = x.tobytes()
            fn = os.path.join(d, "t%04d.wav" % t)
            with open(fn, "wb") as f:
                f.write(struct.pack("<4sI4s4sIHHIIHH4sI", b"RIFF", 36 + len(data), b"WAVE",
                                    b"fmt ", 16, 1, 2, 44100, 44100 * 4, 4, 16, b"data",
                                    len(data)))
                f.write(data)
            files.append(fn)
        go = os.path.join(d, "go")
        ws = []
        for k in range(procs):
            lf = os.path.join(d, "l%d" % k)
            open(lf, "w").write("\n".join(files[k::procs]))
            ws.append(subprocess.Popen([sys.executable, __file__, "--worker", lf, d, go],
                                       stdout=subprocess.PIPE, text=True,
                                       env=dict(os.environ, ATG_ENGINE_STREAMS=os.environ.get(
                                           "ATG_ENGINE_STREAMS", "lazy"))))
        for w in ws:
            json.loads(w.stdout.readline())
        t0 = time.perf_counter()
        open(go, "w").close()
        st = [json.loads(w.stdout.readline()) for w in ws]
        wall = time.perf_counter() - t0
        for w in ws:
            w.wait()
        fr = sum(s["frames"] for s in st)
        print(json.dumps({"procs": procs, "tracks": tracks, "wall_s": round(wall, 3),
                          "frames_per_s": round(fr / wall, 1),
                          "eng_ms_per_call": round(1e3 * sum(s["eng"] for s in st) /
                                                   sum(s["calls"] for s in st), 2),
                          "other_ms_per_track": round(1e3 * sum(s["seconds"] - s["eng"] for s in st)
                                                      / tracks, 2),
                          "last_call_kernel_ms": st[0]["kernel_ms"],
                          "worker0_calls_ms": st[0]["each_ms"]}), flush=True)


if __name__ == "__main__":
    sys.exit(main())
