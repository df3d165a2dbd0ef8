"""Deterministic test signals (restated generators of the reference's
test/test_streams.py and src/decoders/sine.c, plus seeded noise/chirps).
Integer-exact where the reference generators are integer, numpy float64
sin otherwise (rounded to int, stable across machines in practice)."""
import numpy as np

FULL = {8: 0x7F, 16: 0x7FFF, 24: 0x7FFFFF}


def sine_stereo(n, rate, f1, a1, f2, a2, fmult, bps):
    """Sine_Stereo (src/decoders/sine.c:270-285)"""
    fs = FULL[bps]
    d1 = 2 * np.pi / (rate / f1)
    d2 = 2 * np.pi / (rate / f2)
    t1 = np.arange(n) * d1
    t2 = np.arange(n) * d2
    l = ((a1 * np.sin(t1) + a2 * np.sin(t2)) * fs + 0.5).astype(np.int64)
    r = (-(a1 * np.sin(t1 * fmult) + a2 * np.sin(t2 * fmult)) * fs + 0.5).astype(np.int64)
    return np.stack([l, r], 1).reshape(-1).astype(np.int32)


def sine_mono(n, rate, f1, a1, f2, a2, bps):
    fs = FULL[bps]
    t = np.arange(n)
    v = ((a1 * np.sin(t * 2 * np.pi / (rate / f1)) +
          a2 * np.sin(t * 2 * np.pi / (rate / f2))) * fs + 0.5).astype(np.int64)
    return v.astype(np.int32)


def simple_sine(n, max_value, count):
    """one channel of Sine_Simple (src/decoders/sine.c:393-423):
    round(max_value * sin(2 pi (i % count) / count))"""
    i = np.arange(n) % count
    d = max_value * np.sin((np.pi * 2) * i / count)
    return (np.sign(d) * np.floor(np.abs(d) + 0.5)).astype(np.int32)  # C round()


def noise(n, channels, bps, seed):
    rng = np.random.default_rng(seed)
    return rng.integers(-(1 << (bps - 1)), 1 << (bps - 1), n * channels).astype(np.int32)


def tone_noise(n, channels, bps, seed, sigma=8.0):
    """two sines per channel + gaussian noise, clipped"""
    rng = np.random.default_rng(seed)
    fs = FULL[bps]
    t = np.arange(n)
    out = []
    for c in range(channels):
        f1, f2 = rng.uniform(100, 2000), rng.uniform(2000, 12000)
        a1 = rng.uniform(0.05, 0.5)
        a2 = rng.uniform(0.0, 0.85 - a1)
        x = (a1 * np.sin(2 * np.pi * f1 * t / 44100) +
             a2 * np.sin(2 * np.pi * f2 * t / 44100)) * fs
        x = np.round(x + rng.normal(0, sigma, n))
        out.append(np.clip(x, -fs - 1, fs))
    return np.stack(out, 1).reshape(-1).astype(np.int32)


def chirp(n, channels, bps, amp=0.8):
    fs = FULL[bps]
    t = np.arange(n)
    x = np.round(amp * np.sin(2 * np.pi * (20 + 10000.0 * t / max(n, 1)) * t / 44100) * fs)
    return np.repeat(x[:, None], channels, 1).reshape(-1).astype(np.int32)


def wasted_bps16(n):
    """WastedBPS16 (test/test_streams.py:343-370)"""
    i = np.arange(n)
    return np.stack([(i % 2000) << 2, (i % 1000) << 3], 1).reshape(-1).astype(np.int32)


def fsd(pattern, reps, bps):
    """full-scale-deflection patterns (test/test_streams.py:423-448)"""
    hi, lo = (1 << (bps - 1)) - 1, -(1 << (bps - 1))
    return np.array([hi if p > 0 else lo for p in pattern] * reps, dtype=np.int32)


PATTERNS = [[1, -1], [1, 1, -1], [1, -1, -1], [1, -1, 1, -1], [1, -1, -1, 1],
            [1, -1, 1, 1, -1], [1, -1, -1, 1, -1]]

# Generate01-04 (test/test_streams.py:94-116): (samples, channels, bps)
SHORT_STREAMS = [([-32768], 1, 16), ([-32768, 32767], 2, 16),
                 ([-25, 0, 25, 50, 100], 1, 16),
                 ([-25, 500, 0, 400, 25, 300, 50, 200, 100, 100], 2, 16)]


def make(kind, n, channels, bps, seed=1):
    if kind == "sine":
        if channels == 2:
            return sine_stereo(n, 44100, 441.0, 0.61, 661.5, 0.37, 1.3, bps)
        x = sine_mono(n, 44100, 441.0, 0.50, 4410.0, 0.49, bps)
        return np.repeat(x[:, None], channels, 1).reshape(-1)
    if kind == "tone":
        return tone_noise(n, channels, bps, seed)
    if kind == "noise":
        return noise(n, channels, bps, seed)
    if kind == "silence":
        return np.zeros(n * channels, dtype=np.int32)
    if kind == "chirp":
        return chirp(n, channels, bps)
    if kind == "wasted":
        x = noise(n, channels, bps - 4, seed).astype(np.int64) << 4
        return x.astype(np.int32)
    raise ValueError(kind)
