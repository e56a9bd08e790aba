"""Round-2 RTCD shims (include/svtgpu.h) against the reference's own outputs.

Fixtures: tests/golden/lr_stats.bin (svt_av1_compute_stats(_highbd)_c), lr_proj.bin (pixel_proj_error /
get_proj_subspace), md_shims.bin (sub-pixel variance, mse16x16, highbd_8_mse16x16, variance_highbd, nxm SAD),
cdef_shims.bin (svt_cdef_filter_block_8xn_16_avx2, copy_rect8) — written by oracle/ref_harness/gen_golden_lr.c and
gen_golden_shims.c from the reference sources.  Every case of every fixture runs."""
import ctypes

import numpy as np
import pytest

import cdef_cases as cc
import svtgpu

pytestmark = pytest.mark.gpu
P = ctypes.c_void_p
U32 = ctypes.c_uint32


@pytest.fixture(scope="module")
def ctx():
    return svtgpu.Context(0)


def addr(a, off=0):
    return P(a.ctypes.data + off * a.itemsize)


def byteptr(a, off=0):  # CONVERT_TO_BYTEPTR of a uint16 array
    return P((a.ctypes.data + off * 2) >> 1)


def test_compute_stats_shims(ctx):
    L, g = svtgpu.lib(), cc.load("lr_stats.bin")
    for n in range(len(g["meta"])):
        bd, win, w, h, st, _ = (int(x) for x in g["meta"][n])
        d, s = np.ascontiguousarray(g["dgd%d" % n]), np.ascontiguousarray(g["src%d" % n])
        M, H = np.zeros(win * win, np.int64), np.zeros(win ** 4, np.int64)
        o = 4 * st + 4
        if bd == 8:
            d8, s8 = d.astype(np.uint8), s.astype(np.uint8)
            L.svtgpu_av1_compute_stats(win, addr(d8, o), addr(s8, o), 0, w, 0, h, st, st, addr(M), addr(H))
        else:
            L.svtgpu_av1_compute_stats_highbd(win, byteptr(d, o), byteptr(s, o), 0, w, 0, h, st, st, addr(M), addr(H),
                                              bd)
        assert np.array_equal(M, g["M%d" % n]) and np.array_equal(H, g["H%d" % n]), (n, bd, win)


def test_pixel_proj_error_and_subspace_shims(ctx):
    L, g = svtgpu.lib(), cc.load("lr_proj.bin")
    sgr = g["sgr_params"]
    for n in range(len(g["meta"])):
        bd, w, h, eps, xq0, xq1, err, sx0, sx1 = (int(x) for x in g["meta"][n])
        prm = svtgpu.SgrParams((ctypes.c_int32 * 2)(*sgr[eps][:2]), (ctypes.c_int32 * 2)(*sgr[eps][2:]))
        src, dat = np.ascontiguousarray(g["src%d" % n]), np.ascontiguousarray(g["dat%d" % n])
        f0, f1 = np.ascontiguousarray(g["flt0_%d" % n]), np.ascontiguousarray(g["flt1_%d" % n])
        xq = (ctypes.c_int32 * 2)(xq0, xq1)
        sxq = (ctypes.c_int32 * 2)()
        if bd == 8:
            s8, d8 = src.astype(np.uint8), dat.astype(np.uint8)
            got = L.svtgpu_av1_lowbd_pixel_proj_error(addr(s8), w, h, w, addr(d8), w, addr(f0), w, addr(f1), w, xq,
                                                      ctypes.byref(prm))
            L.svtgpu_get_proj_subspace(addr(s8), w, h, w, addr(d8), w, 0, addr(f0), w, addr(f1), w, sxq,
                                       ctypes.byref(prm))
        else:
            got = L.svtgpu_av1_highbd_pixel_proj_error(byteptr(src), w, h, w, byteptr(dat), w, addr(f0), w, addr(f1), w,
                                                       xq, ctypes.byref(prm))
            L.svtgpu_get_proj_subspace(byteptr(src), w, h, w, byteptr(dat), w, 1, addr(f0), w, addr(f1), w, sxq,
                                       ctypes.byref(prm))
        assert got == err, (n, bd, eps, got, err)
        assert (sxq[0], sxq[1]) == (sx0, sx1), (n, bd, eps, tuple(sxq), (sx0, sx1))


def test_md_shims(ctx):
    L, g = svtgpu.lib(), cc.load("md_shims.bin")
    A, B = np.ascontiguousarray(g["A"]), np.ascontiguousarray(g["B"])
    A16, B16 = np.ascontiguousarray(g["A16"]), np.ascontiguousarray(g["B16"])
    S = A.shape[1]
    sse = U32()
    bad = []
    for si, (w, h) in enumerate(svtgpu.MD_SIZES):
        fn = getattr(L, "svtgpu_aom_sub_pixel_variance%dx%d" % (w, h))
        res = g["spv%d" % si]
        for m in range(4):
            off = m * S * S + m * S + 3 * m
            for o in range(64):
                v = fn(addr(A, off), S, o & 7, o >> 3, addr(B, off), S, ctypes.byref(sse))
                if (v, sse.value) != tuple(int(x) for x in res[m * 64 + o]):
                    bad.append(("spv", w, h, m, o))
    assert not bad, bad[:10]
    for n in range(len(g["meta"])):
        m, oy, ox, w, h = (int(x) for x in g["meta"][n])
        want = [int(x) for x in g["res"][n]]
        off = m * S * S + oy * S + ox
        got = [L.svtgpu_aom_mse16x16(addr(A, off), S, addr(B, off), S, ctypes.byref(sse))]
        got.append(sse.value)
        L.svtgpu_aom_highbd_8_mse16x16(byteptr(A16, off), S, byteptr(B16, off), S, ctypes.byref(sse))
        got.append(sse.value)
        got.append(L.svtgpu_aom_variance_highbd(addr(A16, off), S, addr(B16, off), S, w, h, ctypes.byref(sse)))
        got.append(sse.value)
        got.append(L.svtgpu_nxm_sad_kernel(addr(A, off), S, addr(B, off), S, h, w))
        assert L.svtgpu_nxm_sad_kernel_sub_sampled(addr(A, off), S, addr(B, off), S, h, w) == want[5], n
        assert got == want, (n, got, want)


def test_cdef_8xn_and_copy_rect_shims(ctx):
    L, g = svtgpu.lib(), cc.load("cdef_shims.bin")
    for n in range(len(g["meta"])):
        bd, pri, sec, d, pdamp, sdamp, ss = (int(x) for x in g["meta"][n])
        buf = np.full(144 * 12, 0x7F7F, np.uint16)  # CDEF_BSTRIDE buffer, block at row 2, col 2
        for y in range(12):
            buf[y * 144:y * 144 + 12] = g["win"][n][y]
        out = np.full(64, 0xDEAD, np.uint16)
        L.svtgpu_cdef_filter_block_8xn_16(addr(buf, 2 * 144 + 2), pri, sec, d, pdamp, sdamp, bd - 8, addr(out), 8, 8,
                                          ss)
        assert np.array_equal(out, g["out"][n]), (n, bd, ss)
    src = np.ascontiguousarray(g["rect_src"])
    for n in range(len(g["rect_meta"])):
        v, h = (int(x) for x in g["rect_meta"][n])
        dst = np.full(70 * 90, 0xBEEF, np.uint16)
        L.svtgpu_aom_copy_rect8_8bit_to_16bit(addr(dst), 90, addr(src), 90, v, h)
        assert np.array_equal(dst.reshape(70, 90), g["rect_dst"][n]), n
