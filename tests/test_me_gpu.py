"""Open-loop ME SAD parity on the MI355X: the RTCD shims and the frame-level full-pel search against the reference's
golden vectors (tests/golden/me_sad.bin from the reference's own EbMotionEstimation.c / EbComputeSAD_C.c), and the
search at 4K against the CPU oracle on SB subsets (properties of the whole frame: every 64x64 best equals the sum
structure's minimum).  Bit-exact."""
import ctypes

import numpy as np
import pytest

import me_cases as mc
import oracle
import svtgpu

pytestmark = pytest.mark.gpu
P = lambda a: ctypes.c_void_p(a.ctypes.data)


@pytest.fixture(scope="module")
def ctx():
    return svtgpu.Context(0)


@pytest.fixture(scope="module")
def g():
    return mc.golden()


def luma_frame(ctx, y):
    h, w = y.shape
    f = svtgpu.Frame(ctx, w, h, 8)
    f.upload([y, np.zeros((h // 2, w // 2), np.uint8), np.zeros((h // 2, w // 2), np.uint8)])
    return f


def test_me_search_golden(ctx, g):
    for src, refs, origin, saw, sah, sub, sad, mv in mc.frames(g):
        h, w = src.shape
        me = svtgpu.MeBatch(ctx, w, h, len(refs))
        me.set_origins(origin)
        me.search(luma_frame(ctx, src), [luma_frame(ctx, r) for r in refs], saw, sah, sub)
        gs, gm = me.read()
        np.testing.assert_array_equal(gs, sad, err_msg="sad %dx%d sa %dx%d sub %d" % (w, h, saw, sah, sub))
        np.testing.assert_array_equal(gm, mv, err_msg="mv %dx%d sa %dx%d sub %d" % (w, h, saw, sah, sub))


def test_all_sad_and_eight_sad_shims_golden(g):
    L = svtgpu.lib()
    srcs, wins, ins, e16s, e32s, mvs = g["all_src"], g["all_win"], g["all_in"], g["all_e16"], g["all_e32"], g["all_mv"]
    for n in range(len(mvs)):
        s = np.ascontiguousarray(srcs[64 * n:64 * n + 64])
        r = np.ascontiguousarray(wins[80 * n:80 * n + 80])
        mv, sub = int(mvs[n][0]), int(mvs[n][1])
        b, m = ins[2 * n].copy(), ins[2 * n + 1].copy()
        e16 = np.zeros((16, 8), np.uint32)
        e8 = np.zeros((64, 8), np.uint32)
        e32 = np.zeros((4, 8), np.uint32)
        L.svtgpu_ext_all_sad_calculation_8x8_16x16(P(s), 80, P(r), 80, mv, P(b), P(b[64:]), P(m), P(m[64:]), P(e16),
                                                   P(e8), sub)
        L.svtgpu_ext_eight_sad_calculation_32x32_64x64(P(e16), P(b[80:]), P(b[84:]), P(m[80:]), P(m[84:]), mv, P(e32))
        np.testing.assert_array_equal(e16, e16s[16 * n:16 * n + 16], err_msg=str(n))
        np.testing.assert_array_equal(e32, e32s[4 * n:4 * n + 4], err_msg=str(n))
        np.testing.assert_array_equal(b, g["all_out_sad%d" % n], err_msg=str(n))
        np.testing.assert_array_equal(m, g["all_out_mv%d" % n], err_msg=str(n))


def test_single_point_shims_golden(g):
    """svt_ext_sad_calculation_8x8_16x16 + _32x32_64x64 at x .. x + 7 (the single-point path of the search) reach the
    eight-point path's golden bests: the strict "<" updates of every entry see the same SADs in the same order."""
    L = svtgpu.lib()
    zoff = [0, 1, 4, 5, 2, 3, 6, 7, 8, 9, 12, 13, 10, 11, 14, 15]
    srcs, wins, ins, mvs = g["all_src"], g["all_win"], g["all_in"], g["all_mv"]
    for n in range(0, len(mvs), 3):
        s = np.ascontiguousarray(srcs[64 * n:64 * n + 64])
        r = np.ascontiguousarray(wins[80 * n:80 * n + 80])
        mv0, sub = int(mvs[n][0]), int(mvs[n][1])
        b, m = ins[2 * n].copy(), ins[2 * n + 1].copy()
        for p in range(8):
            x = ((mv0 & 0xFFFF) + p) & 0xFFFF
            mv = (mv0 & 0xFFFF0000) | x
            s16 = np.zeros(16, np.uint32)
            s8 = np.zeros(4, np.uint32)
            s32 = np.zeros(4, np.uint32)
            for by in range(4):
                for bx in range(4):
                    q = zoff[4 * by + bx]
                    sp = ctypes.c_void_p(s.ctypes.data + 16 * by * 80 + 16 * bx)
                    rp = ctypes.c_void_p(r.ctypes.data + 16 * by * 80 + 16 * bx + p)
                    L.svtgpu_ext_sad_calculation_8x8_16x16(sp, 80, rp, 80, P(b[4 * q:]), P(b[64 + q:]), P(m[4 * q:]),
                                                           P(m[64 + q:]), mv, P(s16[q:]), P(s8), sub)
            L.svtgpu_ext_sad_calculation_32x32_64x64(P(s16), P(b[80:]), P(b[84:]), P(m[80:]), P(m[84:]), mv, P(s32))
        np.testing.assert_array_equal(b, g["all_out_sad%d" % n], err_msg=str(n))
        np.testing.assert_array_equal(m, g["all_out_mv%d" % n], err_msg=str(n))


def test_sad_loop_shim_golden(g):
    L = svtgpu.lib()
    for s, r, meta in mc.loop_cases(g):
        bw, bh, saw, sah, ss, rs, srr, skip, best, c = meta
        b, xc, yc = ctypes.c_uint64(0), ctypes.c_int16(-1), ctypes.c_int16(-1)
        L.svtgpu_sad_loop_kernel(P(s), ss, P(r), rs, bh, bw, ctypes.byref(b), ctypes.byref(xc), ctypes.byref(yc), srr,
                                 skip, saw, sah)
        assert b.value == best, meta
        if best < 0xffffff:
            assert (xc.value & 0xFFFF) | ((yc.value & 0xFFFF) << 16) == c & 0xFFFFFFFF, meta


@pytest.mark.parametrize("saw,sah,sub", [(32, 32, 0), (45, 11, 1)])
def test_me_search_4k_vs_oracle(ctx, saw, sah, sub):
    """3840x2160, 4 references, random origins reaching past the frame edges: SB subsets against the oracle (first,
    middle and last rows of blocks), and on the whole frame the hierarchy's consistency (a 64x64 best is never above
    the SAD of its own MV's 8x8 sums, which the oracle subsets check exactly)."""
    import synth
    W, H, nref = 3840, 2160, 4
    rng = np.random.default_rng(7 + saw)
    src = synth.frame_pair(W, H, 8, seed=0x5EED0011)[0][0]
    refs = [synth.frame_pair(W, H, 8, seed=0x5EED0012 + 5 * k)[0][0] for k in range(nref)]
    nsb = ((W + 63) // 64) * ((H + 63) // 64)
    origin = rng.integers(-48, 24, size=(nsb, nref, 2)).astype(np.int16)
    me = svtgpu.MeBatch(ctx, W, H, nref)
    me.set_origins(origin)
    me.search(luma_frame(ctx, src), [luma_frame(ctx, r) for r in refs], saw, sah, sub)
    gs, gm = me.read()
    assert gs.shape == (nsb, nref, 85)
    assert (gs < 128 * 128 * 255).all()
    for b, e in ((0, 6), (nsb // 2, nsb // 2 + 6), (nsb - 6, nsb)):
        osad, omv = oracle.me_search(src, refs, origin, saw, sah, sub, sb_range=(b, e))
        np.testing.assert_array_equal(gs[b:e], osad, err_msg="sad sbs %d-%d" % (b, e))
        np.testing.assert_array_equal(gm[b:e], omv, err_msg="mv sbs %d-%d" % (b, e))
    # every best MV lies inside the searched area
    mx = (gm & 0xFFFF).astype(np.int32)
    mx = np.where(mx >= 32768, mx - 65536, mx)
    my = (gm >> 16).astype(np.int32)
    my = np.where(my >= 32768, my - 65536, my)
    ox, oy = origin[..., 0:1].astype(np.int32), origin[..., 1:2].astype(np.int32)
    assert ((mx >= ox) & (mx < ox + saw) & (my >= oy) & (my < oy + sah)).all()


def test_pme_sad_loop_shim_golden(g):
    """svt_pme_sad_loop_kernel (MD full-pel search, SAD + MV rate of every MV_COST_TYPE) against the reference's own
    results on 40 golden calls: block sizes 4..128, steps 1..3, search areas not a multiple of 8."""
    L = svtgpu.lib()
    for p, keep, s, r, m in mc.pme_cases(g):
        bw, bh, saw, sah, step, ss, rs = m[:7]
        best, bx, by = ctypes.c_uint32(m[10] & 0xFFFFFFFF), ctypes.c_int16(111), ctypes.c_int16(-111)
        L.svtgpu_pme_sad_loop_kernel(ctypes.byref(p), P(s), ss, P(r), rs, bh, bw, ctypes.byref(best),
                                     ctypes.byref(bx), ctypes.byref(by), m[13], m[14], saw, sah, step, m[15], m[16])
        assert (best.value, bx.value, by.value) == (m[17] & 0xFFFFFFFF, m[18], m[19]), m
