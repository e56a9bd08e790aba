"""Deterministic synthetic 4:2:0 inputs (BASELINE.md §3 / SURVEY.md §8d).

source = clip(smooth 2-D gradient + oriented sinusoid texture (random angle per 64x64 block, so
CDEF directions vary) + Gaussian noise sigma = 3*2^(bd-8));
recon  = clip(source + per-8x8 DC offset U(-q/2, q/2) + ringing noise U(-q, q)), q = 6*2^(bd-8).
Values in [0, 2^bd - 1]; uint8 for 8-bit, uint16 for 10-bit.  Chroma uses the same generator at half
resolution.  seed = 0x5EED0000 + config number by convention.
"""
import numpy as np


def _plane(rng, h, w, bd):
    maxv = (1 << bd) - 1
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float32)
    base = (0.25 + 0.5 * (xx / max(w, 1)) * 0.6 + 0.5 * (yy / max(h, 1)) * 0.4) * maxv
    nbh, nbw = (h + 63) // 64, (w + 63) // 64
    ang = rng.uniform(0, np.pi, size=(nbh, nbw)).astype(np.float32)
    freq = rng.uniform(0.15, 0.6, size=(nbh, nbw)).astype(np.float32)
    amp = rng.uniform(0.02, 0.12, size=(nbh, nbw)).astype(np.float32) * maxv
    A = np.repeat(np.repeat(ang, 64, 0), 64, 1)[:h, :w]
    F = np.repeat(np.repeat(freq, 64, 0), 64, 1)[:h, :w]
    M = np.repeat(np.repeat(amp, 64, 0), 64, 1)[:h, :w]
    tex = M * np.sin(F * (xx * np.cos(A) + yy * np.sin(A)))
    noise = rng.normal(0.0, 3.0 * (1 << (bd - 8)), size=(h, w)).astype(np.float32)
    return np.clip(np.rint(base + tex + noise), 0, maxv)


def _coded(rng, src, bd):
    h, w = src.shape
    maxv = (1 << bd) - 1
    q = 6.0 * (1 << (bd - 8))
    dc = rng.uniform(-q / 2, q / 2, size=((h + 7) // 8, (w + 7) // 8)).astype(np.float32)
    DC = np.repeat(np.repeat(dc, 8, 0), 8, 1)[:h, :w]
    ring = rng.uniform(-q, q, size=(h, w)).astype(np.float32)
    return np.clip(np.rint(src + DC + ring), 0, maxv)


def frame_pair(width, height, bit_depth, seed):
    """Returns (source_planes, recon_planes), each a list [Y, U, V] of 2-D arrays."""
    rng = np.random.Generator(np.random.PCG64(seed))
    dt = np.uint16 if bit_depth > 8 else np.uint8
    src, rec = [], []
    for p in range(3):
        h, w = (height, width) if p == 0 else (height // 2, width // 2)
        s = _plane(rng, h, w, bit_depth)
        r = _coded(rng, s, bit_depth)
        src.append(s.astype(dt))
        rec.append(r.astype(dt))
    return src, rec


# ---------------------------------------------------------------------------------------------
# integer-only generator (bit-identical on every host): the inputs of the reference-pinned pipeline cases
# (tests/pipeline_cases.py; tests/golden/pipe_*.npz hold the reference's outputs on them) and of bench.py
# ---------------------------------------------------------------------------------------------
def _plane_int(rng, h, w, bd):
    """Gradient + oriented triangle-wave texture per 64x64 block + uniform noise, integers only."""
    maxv = (1 << bd) - 1
    yy, xx = np.mgrid[0:h, 0:w].astype(np.int64)
    base = maxv // 4 + (xx * (maxv // 3)) // max(w, 1) + (yy * (maxv // 5)) // max(h, 1)
    nbh, nbw = (h + 63) // 64, (w + 63) // 64
    dirs = np.array([(1, 0), (0, 1), (1, 1), (1, -1), (2, 1), (1, 2), (2, -1), (1, -2)], np.int64)
    d = dirs[rng.integers(0, 8, size=(nbh, nbw))]
    period = rng.integers(3, 13, size=(nbh, nbw)).astype(np.int64)
    amp = rng.integers(maxv // 60 + 1, maxv // 8 + 2, size=(nbh, nbw)).astype(np.int64)

    def up(a):
        return np.repeat(np.repeat(a, 64, 0), 64, 1)[:h, :w]

    dx, dy, P, A = up(d[..., 0]), up(d[..., 1]), up(period), up(amp)
    t = np.mod(xx * dx + yy * dy, 2 * P)
    tex = A * (np.abs(t - P) * 2 - P) // P
    k = 3 << (bd - 8)
    noise = rng.integers(-k, k + 1, size=(h, w))
    return np.clip(base + tex + noise, 0, maxv)


def _coded_int(rng, src, bd):
    h, w = src.shape
    maxv = (1 << bd) - 1
    q = 6 << (bd - 8)
    dc = rng.integers(-q // 2, q // 2 + 1, size=((h + 7) // 8, (w + 7) // 8))
    ring = rng.integers(-q, q + 1, size=(h, w))
    return np.clip(src + np.repeat(np.repeat(dc, 8, 0), 8, 1)[:h, :w] + ring, 0, maxv)


def frame_pair_int(width, height, bit_depth, seed):
    """(source_planes, recon_planes) from the integer generator (PCG64 integer draws, integer arithmetic)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    dt = np.uint16 if bit_depth > 8 else np.uint8
    src, rec = [], []
    for p in range(3):
        ph, pw = (height, width) if p == 0 else (height // 2, width // 2)
        s = _plane_int(rng, ph, pw, bit_depth)
        src.append(s.astype(dt))
        rec.append(_coded_int(rng, s, bit_depth).astype(dt))
    return src, rec


def block_mask(width, height, seed, p_skip=0.0):
    """Per-8x8 'filter this block' mask (1 = listed); p_skip = probability a block is skipped."""
    rng = np.random.Generator(np.random.PCG64(seed ^ 0xB10C))
    m = (rng.random(((height + 7) // 8, (width + 7) // 8)) >= p_skip).astype(np.uint8)
    return m


def mode_info(width, height, seed):
    """Deblocking mode-info grid for the benchmark: 16x16 non-skip inter blocks
    (LAST_FRAME, NEWMV), transform size hashed per block from {16, 8, 4} (tx_depth 0/1/2).
    Returns a structured array [mi_rows][mi_cols] with svtgpu.LF_MI_DTYPE."""
    from svtgpu import LF_MI_DTYPE
    mr, mc = ((height + 7) & ~7) >> 2, ((width + 7) & ~7) >> 2
    mi = np.zeros((mr, mc), LF_MI_DTYPE)
    by, bx = np.mgrid[0:mr, 0:mc] // 4
    h = (by * 0x9E3779B1 + bx * 0x85EBCA77 + seed) & 0xFFFFFFFF
    h = ((h ^ (h >> 15)) * 0x2C1B3C6D) & 0xFFFFFFFF
    mi["bsize"] = 6           # BLOCK_16X16
    mi["tx_depth"] = (h >> 7) % 3
    mi["skip"] = 0
    mi["ref_frame0"] = 1      # LAST_FRAME
    mi["mode"] = 16           # NEWMV
    return mi
