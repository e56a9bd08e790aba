"""Mode-decision distortion parity on the MI355X (SAD / SSE / variance): RTCD shims vs the reference's
golden vectors, the batched kernel vs the CPU oracle.  Bit-exact."""
import ctypes

import numpy as np
import pytest

import md_cases as mc
import oracle
import svtgpu
import synth

pytestmark = pytest.mark.gpu
P = lambda a: ctypes.c_void_p(a.ctypes.data)


@pytest.fixture(scope="module")
def ctx():
    return svtgpu.Context(0)


def test_md_shims_golden(ctx):
    L = svtgpu.lib()
    g = mc.golden()
    for si, (w, h) in enumerate(mc.MD_SIZES):
        res = g["s%d_res" % si]
        for c in range(res.shape[0]):
            s16, r16, s8, r8 = mc.case(g, si, c)
            st = s16.shape[1]
            sse = ctypes.c_uint32()
            assert getattr(L, "svtgpu_aom_sad%dx%d" % (w, h))(P(s8), st, P(r8), st) == res[c][0], (w, h, c)
            assert getattr(L, "svtgpu_aom_variance%dx%d" % (w, h))(P(s8), st, P(r8), st, ctypes.byref(sse)) == res[c][1]
            assert sse.value == res[c][2]
            # highbd variance takes CONVERT_TO_BYTEPTR-encoded pointers (address >> 1)
            a8, b8 = ctypes.c_void_p(s16.ctypes.data >> 1), ctypes.c_void_p(r16.ctypes.data >> 1)
            assert getattr(L, "svtgpu_aom_highbd_10_variance%dx%d" % (w, h))(a8, st, b8, st, ctypes.byref(sse)) \
                == res[c][3], (w, h, c)
            assert sse.value == res[c][4]
            assert L.svtgpu_sad_16b_kernel(P(s16), st, P(r16), st, h, w) == res[c][5]
            refs = (ctypes.c_void_p * 4)(*[r8.ctypes.data + o for o in (0, 1, st, 3 * st + 2)])
            out4 = np.zeros(4, np.uint32)
            getattr(L, "svtgpu_aom_sad%dx%dx4d" % (w, h))(P(s8), st, refs, st, P(out4))
            assert list(out4) == list(res[c][6:10])
            e8 = L.svtgpu_aom_sse(P(s8), st, P(r8), st, w, h)
            assert e8 & 0xFFFFFFFF == res[c][10]
            assert L.svtgpu_spatial_full_distortion_kernel(P(s8), 0, st, P(r8), 0, st, w, h) == e8
            e16 = L.svtgpu_aom_highbd_sse(P(s16), st, P(r16), st, w, h)
            assert (e16 >> 4) & 0xFFFFFFFF == res[c][11]
            assert L.svtgpu_full_distortion_kernel16_bits(P(s16), 0, st, P(r16), 0, st, w, h) == e16


BATCH_CASES = [(200, 136, 8, 1, 3), (320, 256, 10, 7, 4), (1920, 1080, 10, 7, 5), (136, 72, 10, 2, 6)]


@pytest.mark.parametrize("w,h,bd,nref,seed", BATCH_CASES)
def test_md_batch_vs_oracle(ctx, w, h, bd, nref, seed):
    src, _ = synth.frame_pair(w, h, bd, seed=0x5EED0500 + seed)
    refs = mc.ref_frames(w, h, bd, nref, 0x5EED0500 + seed)
    mv = mc.mvs(w, h, nref, seed, rng_max=24)
    want = oracle.md_dist_batch(src[0], refs, bd, mv)
    S = svtgpu.Frame(ctx, w, h, bd)
    S.upload(src)
    R = []
    for r in refs:
        f = svtgpu.Frame(ctx, w, h, bd)
        f.upload([r, src[1], src[2]])
        R.append(f)
    b = svtgpu.MdBatch(ctx, w, h, nref)
    b.set_mvs(mv)
    b.run(S, R)
    got = b.read()
    assert np.array_equal(got, want)
    # a sub-range of SBs (multi-GPU row bands) writes exactly its rows
    b2 = svtgpu.MdBatch(ctx, w, h, nref)
    b2.set_mvs(mv)
    half = b2.nsb // 2
    b2.run(S, R, half, b2.nsb)
    assert np.array_equal(b2.read(half, b2.nsb), want[half:])


def test_md_layout(ctx):
    w, h, o = svtgpu.md_layout()
    assert list(zip(w, h)) == oracle.MD_SHAPES
    assert o[-1] + 4096 // (w[-1] * h[-1]) == svtgpu.MD_BLOCKS


def test_md_batch_8k_10bit(ctx):
    """Config 5's frame on one GPU: 7680x4320 10-bit, 7 references, MVs reaching past the frame edges.  SB subsets
    (first, middle and last SB rows' ends) against the oracle; on the whole frame, the shape hierarchy: for every SB
    and reference the SADs of each shape's blocks sum to the 64x64 block's (the SSEs to within their rounding), and
    variance <= SSE."""
    import time
    w, h, bd, nref = 7680, 4320, 10, 7
    t0 = time.time()
    src, _ = synth.frame_pair(w, h, bd, seed=0x5EED0580)
    rng = np.random.default_rng(0x5EED0581)  # references: shifted source plus noise (fast at 8K)
    refs = [np.clip(np.roll(src[0].astype(np.int32), (3 * k - 9, 5 - 2 * k), axis=(0, 1)) +
                    rng.integers(-24, 25, size=(h, w)), 0, 1023).astype(np.uint16) for k in range(nref)]
    mv = mc.mvs(w, h, nref, 8, rng_max=40)
    S = svtgpu.Frame(ctx, w, h, bd)
    S.upload(src)
    R = []
    for r in refs:
        f = svtgpu.Frame(ctx, w, h, bd)
        f.upload([r, src[1], src[2]])
        R.append(f)
    b = svtgpu.MdBatch(ctx, w, h, nref)
    assert b.nsb == 120 * 68
    b.set_mvs(mv)
    b.run(S, R)
    got = b.read()
    print("8K MD batch: setup + run + read %.1f s" % (time.time() - t0))
    for lo, hi in ((0, 4), (b.nsb // 2 - 2, b.nsb // 2 + 2), (b.nsb - 4, b.nsb)):
        want = oracle.md_dist_batch(src[0], refs, bd, mv, sb_range=(lo, hi))
        assert np.array_equal(got[lo:hi], want), (lo, hi)
    wl, hl, off = svtgpu.md_layout()
    whole = int(off[[s for s in range(len(wl)) if wl[s] == 64 and hl[s] == 64][0]])  # the 64x64 block
    g64 = got.astype(np.uint64)
    for s in range(len(wl)):
        n = 4096 // (wl[s] * hl[s])
        tot = g64[:, :, 0, off[s]:off[s] + n].sum(axis=-1)  # SAD: additive over a shape's tiling of the SB
        assert np.array_equal(tot, g64[:, :, 0, whole]), (wl[s], hl[s])
        # 10-bit SSE: each block's is rounded (>> 4, highbd_10_variance), so the sum is within n / 2 of the whole's
        d = g64[:, :, 1, off[s]:off[s] + n].sum(axis=-1).astype(np.int64) - g64[:, :, 1, whole].astype(np.int64)
        assert (np.abs(d) <= n // 2 + 1).all(), (wl[s], hl[s], int(np.abs(d).max()))
    assert (got[:, :, 2, :] <= got[:, :, 1, :]).all()
