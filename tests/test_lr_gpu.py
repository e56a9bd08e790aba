"""Loop-restoration parity on the MI355X: RTCD shims vs the reference's golden vectors, the frame apply
vs the reference's whole-frame golden outputs and vs the CPU oracle.  Bit-exact."""
import ctypes

import numpy as np
import pytest

import cdef_cases as cc
import lr_cases as lc
import oracle
import svtgpu
import synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    return svtgpu.Context(0)


def _at(a, y, x, enc=False):
    addr = a.ctypes.data + (y * a.shape[1] + x) * a.itemsize
    return ctypes.c_void_p(addr >> 1 if enc else addr)


def test_wiener_shims_golden(ctx):
    L = svtgpu.lib()
    g = cc.load("lr_wiener.bin")
    for n in range(len(g["meta"])):
        bd, w, h = (int(x) for x in g["meta"][n])
        fx, fy = (np.ascontiguousarray(g["taps"][n][k * 8:(k + 1) * 8]).copy() for k in range(2))
        inp = g["in%d" % n].copy()
        r0, r1 = oracle.wiener_round(bd)
        cp = svtgpu.ConvolveParams(round_0=r0, round_1=r1)
        if bd == 8:
            i8 = inp.astype(np.uint8)
            o8 = np.zeros((h, w), np.uint8)
            L.svtgpu_av1_wiener_convolve_add_src(_at(i8, 3, 3), i8.shape[1], ctypes.c_void_p(o8.ctypes.data), w,
                                                 ctypes.c_void_p(fx.ctypes.data), ctypes.c_void_p(fy.ctypes.data),
                                                 w, h, ctypes.byref(cp))
            got = o8.astype(np.uint16)
        else:
            got = np.zeros((h, w), np.uint16)
            L.svtgpu_av1_highbd_wiener_convolve_add_src(_at(inp, 3, 3, True), inp.shape[1], _at(got, 0, 0, True), w,
                                                        ctypes.c_void_p(fx.ctypes.data),
                                                        ctypes.c_void_p(fy.ctypes.data), w, h, ctypes.byref(cp), bd)
        assert np.array_equal(got, g["out%d" % n]), (n, bd, w, h)


def test_sgr_shims_golden(ctx):
    L = svtgpu.lib()
    g = cc.load("lr_sgr.bin")
    for n in range(len(g["meta"])):
        bd, w, h, eps, x0, x1 = (int(x) for x in g["meta"][n])
        inp = g["in%d" % n].copy()
        hb = bd > 8
        src = inp if hb else inp.astype(np.uint8)
        f0, f1 = np.zeros((h, w), np.int32), np.zeros((h, w), np.int32)
        L.svtgpu_av1_selfguided_restoration(_at(src, 3, 3, hb), w, h, src.shape[1], ctypes.c_void_p(f0.ctypes.data),
                                            ctypes.c_void_p(f1.ctypes.data), w, eps, bd, int(hb))
        if eps < 10 or eps >= 14:
            assert np.array_equal(f0, g["flt0_%d" % n]), (n, eps)
        if eps < 14:
            assert np.array_equal(f1, g["flt1_%d" % n]), (n, eps)
        out = np.zeros((h, w), np.uint16 if hb else np.uint8)
        xqd = np.array([x0, x1], np.int32)
        L.svtgpu_apply_selfguided_restoration(_at(src, 3, 3, hb), w, h, src.shape[1], eps,
                                              ctypes.c_void_p(xqd.ctypes.data), _at(out, 0, 0, hb), w, None, bd,
                                              int(hb))
        assert np.array_equal(out.astype(np.uint16), g["out%d" % n]), (n, eps)


def _coded(planes, seed):
    """Crop-size planes (the restored area) inside the 8-aligned coded frame the device stages work on: the samples
    past the crop are random, so a read of them would show in the results."""
    h, w = planes[0].shape
    w8, h8 = (w + 7) & ~7, (h + 7) & ~7
    if (w8, h8) == (w, h):
        return planes
    r = np.random.default_rng(seed)
    out = []
    for p, a in enumerate(planes):
        pw, ph = (w8, h8) if p == 0 else (w8 // 2, h8 // 2)
        b = r.integers(0, int(a.max()) + 1, (ph, pw)).astype(a.dtype)
        b[:a.shape[0], :a.shape[1]] = a
        out.append(b)
    return out


def _gpu_apply(ctx, dlf, cdef, bd, frame_type, unit_size, units):
    h, w = cdef[0].shape  # the crop size; the frames are the coded size
    dlf8, cdef8 = _coded(dlf, 1), _coded(cdef, 2)
    D, C, O = (svtgpu.Frame(ctx, cdef8[0].shape[1], cdef8[0].shape[0], bd) for _ in range(3))
    D.upload(dlf8)
    C.upload(cdef8)
    st = svtgpu.LrState(ctx, w, h, unit_size)
    for p in range(3):
        st.set_units(p, units[p])
    st.apply(D, C, O, frame_type)
    got = O.download()
    for p in range(3):  # past the crop the output keeps the CDEF samples
        ph, pw = cdef[p].shape
        m = np.ones(got[p].shape, bool)
        m[:ph, :pw] = False
        assert np.array_equal(got[p][m], cdef8[p][m]), p
    return [got[p][:cdef[p].shape[0], :cdef[p].shape[1]] for p in range(3)]


@pytest.mark.parametrize("case", list(range(9)))
def test_lr_frame_golden(ctx, case):
    """The reference's svt_av1_loop_restoration_filter_frame outputs (gen_golden_lr.c), cases 6-8 at crop sizes that
    are not multiples of 8 (odd chroma widths / heights)."""
    c = list(lc.frame_cases())[case]
    got = _gpu_apply(ctx, c["dlf"], c["cdef"], c["bd"], c["frame_type"], c["unit_size"], c["units"])
    for p in range(3):
        assert np.array_equal(got[p], c["out"][p]), (c["name"], p)


def _crop_pair(w, h, bd, seed):
    """A synthetic (source, recon) pair at a crop size: generated at the coded size and cut to the crop."""
    src, rec = synth.frame_pair((w + 7) & ~7, (h + 7) & ~7, bd, seed=seed)
    cut = lambda planes: [a[:(h if p == 0 else (h + 1) // 2), :(w if p == 0 else (w + 1) // 2)] for p, a in enumerate(planes)]
    return cut(src), cut(rec)


# the last two: crop sizes of a 1366 x 766 picture (683 x 383 chroma) and 330 x 182 (165 x 91)
LR_CASES = [(640, 360, 10, 64, 1), (1920, 1080, 8, 128, 2), (392, 232, 8, 256, 3), (3840, 2160, 10, 256, 4),
            (1366, 766, 10, 64, 5), (330, 182, 8, 128, 6)]


@pytest.mark.parametrize("w,h,bd,usize,seed", LR_CASES)
def test_lr_frame_vs_oracle(ctx, w, h, bd, usize, seed):
    src, rec = _crop_pair(w, h, bd, seed=0x5EED0700 + seed)
    dlf = rec
    cdef = [np.clip(p.astype(np.int32) + ((src[i].astype(np.int32) - p) >> 2), 0, (1 << bd) - 1).astype(p.dtype)
            for i, p in enumerate(rec)]
    unit_size = [usize, usize >> 1, usize >> 1]
    units = []
    for p in range(3):
        pw, ph = (w, h) if p == 0 else ((w + 1) // 2, (h + 1) // 2)
        n = oracle.lr_units(unit_size[p], pw) * oracle.lr_units(unit_size[p], ph)
        units.append(lc.random_units(n, seed * 10 + p, chroma=p > 0))
    ft = [1, 1, 1]
    want = oracle.lr_apply_frame(dlf, cdef, bd, ft, unit_size, units)
    got = _gpu_apply(ctx, dlf, cdef, bd, ft, unit_size, units)
    for p in range(3):
        assert np.array_equal(got[p], want[p]), p


# ------------------------------------------------------------------ search
def _gpu_search(ctx, rec, src, bd, unit_size, ctrls):
    h, w = rec[0].shape  # the crop size; the frames are the coded size
    rec8, src8 = _coded(rec, 3), _coded(src, 4)
    R, S = (svtgpu.Frame(ctx, rec8[0].shape[1], rec8[0].shape[0], bd) for _ in range(2))
    R.upload(rec8)
    S.upload(src8)
    st = svtgpu.LrState(ctx, w, h, unit_size)
    ft, recs = st.search(R, S, ctrls, records=True)
    return st, R, ft, recs


@pytest.mark.parametrize("case", list(range(len(list(lc.search_cases())))))
def test_lr_search_golden(ctx, case):
    """The reference's restoration_seg_search + rest_finish_search records (gen_golden_lr.c), cases 6-9 at crop sizes
    that are not multiples of 8, cases 10-13 with one filter type searched for luma only (the finish's shared
    RestUnitSearchInfo array: c13's chroma takes a Wiener unit from luma's entry).  The RD finish runs on the device
    (lr_fin_*_kernel) unless SVTGPU_LR_FINISH=host."""
    c = list(lc.search_cases())[case]
    st, R, ft, recs = _gpu_search(ctx, c["rec"], c["src"], c["bd"], c["unit_size"], c["ctrls"])
    lc.compare_search(ft, c["units"], recs, c)  # frame types + per-unit records vs the reference
    # the picked units stay in the state: applying them must equal applying the reference's picked units
    h, w = R.height, R.width
    rec8 = _coded(c["rec"], 3)
    D, O = svtgpu.Frame(ctx, w, h, c["bd"]), svtgpu.Frame(ctx, w, h, c["bd"])
    D.upload(rec8)
    st.apply(D, R, O, ft)
    want = oracle.lr_apply_frame(c["rec"], c["rec"], c["bd"], ft, c["unit_size"], c["units"])
    got = O.download()
    for p in range(3):
        assert np.array_equal(got[p][:want[p].shape[0], :want[p].shape[1]], want[p]), (c["name"], p)


LR_SEARCH_CASES = [(320, 192, 10, 64, 1, 1, 5), (640, 360, 8, 128, 1, 1, 6), (1920, 1080, 10, 256, 1, 1, 7),
                   (512, 288, 10, 128, 3, 2, 8), (328, 184, 10, 64, 1, 1, 9), (264, 152, 8, 64, 2, 3, 10),
                   (1366, 766, 10, 64, 1, 1, 11), (330, 182, 8, 64, 2, 3, 12), (1918, 1078, 10, 256, 1, 1, 13)]


@pytest.mark.parametrize("w,h,bd,usize,wn,sg,seed", LR_SEARCH_CASES)
def test_lr_search_vs_oracle(ctx, w, h, bd, usize, wn, sg, seed):
    src, rec = _crop_pair(w, h, bd, seed=0x5EED0800 + seed)
    ctrls = oracle.lr_controls(wn, sg, rdmult=6000 + seed * 1000, switchable=(300, 700, 900), wiener=(250, 800),
                               sgrproj=(250, 900))
    unit_size = [usize, usize >> 1, usize >> 1]
    want_ft, want_units, want_recs = oracle.lr_search_frame(rec, src, bd, unit_size, ctrls)
    st, R, ft, recs = _gpu_search(ctx, rec, src, bd, unit_size, ctrls)
    assert ft == want_ft
    for p in range(3):
        for k in ("sse",):
            np.testing.assert_array_equal(recs[p][k], want_recs[p][k], err_msg="plane %d %s" % (p, k))
        np.testing.assert_array_equal(recs[p]["sgrproj"], want_recs[p]["sgrproj"])
        ok = recs[p]["sse"][:, 1] != np.iinfo(np.int64).max
        np.testing.assert_array_equal(recs[p]["wiener"][ok], want_recs[p]["wiener"][ok])
    # the searched units drive the apply: compare the restored frame with the oracle apply of the oracle's units
    D, O = svtgpu.Frame(ctx, R.width, R.height, bd), svtgpu.Frame(ctx, R.width, R.height, bd)
    D.upload(_coded(rec, 3))
    st.apply(D, R, O, ft)
    want = oracle.lr_apply_frame(rec, rec, bd, ft, unit_size, want_units)
    got = O.download()
    for p in range(3):
        assert np.array_equal(got[p][:want[p].shape[0], :want[p].shape[1]], want[p]), p


@pytest.mark.parametrize("nb", [2, 3])
def test_lr_search_units_bands(ctx, nb):
    """svtgpu_lr_search_units over unit-row bands + svtgpu_lr_finish_plane == the whole-frame search (the
    multi-GPU split of bench.py, run as bands on one device)."""
    w, h, bd, usize = 640, 360, 10, 64
    src, rec = synth.frame_pair(w, h, bd, seed=0x5EED0A00 + nb)
    ctrls = oracle.lr_controls(1, 1, rdmult=7000, switchable=(300, 700, 900), wiener=(250, 800), sgrproj=(250, 900))
    unit_size = [usize, usize >> 1, usize >> 1]
    st, R, ft, recs = _gpu_search(ctx, rec, src, bd, unit_size, ctrls)
    S = svtgpu.Frame(ctx, w, h, bd)
    S.upload(src)
    merged = None
    for r in range(nb):
        rb, re_ = svtgpu.lr_unit_rows(st.units, nb, r)
        merged = st.search_units(R, S, ctrls, rb, re_, merged)
    want_ft, want_units, _ = oracle.lr_search_frame(rec, src, bd, unit_size, ctrls)
    for p in range(3):
        assert merged[p].tobytes() == recs[p].tobytes(), p
        fin_ft, fin_units = svtgpu.lr_finish_plane(ctrls, p, merged[p])
        assert fin_ft == ft[p] == want_ft[p]
        assert fin_units.tobytes() == want_units[p].tobytes(), p


@pytest.mark.parametrize("case", ["mini10", "mini8", "sb128_10", "mini8c", "c3_4k10"])
def test_wiener_stats_mfma_vs_reference(ctx, case):
    """The MFMA Wiener statistics (wiener_stats_kernel: the i8 hi/lo Gram on v_mfma_i32_16x16x64_i8) compared entry by
    entry with the reference's own svt_av1_compute_stats(_highbd)_c, which gen_golden_pipe records for every unit its
    restoration_seg_search visits (M and H of each call; SHA-256 of the whole 4K set).  The compute_stats RTCD shim
    runs the search's kernel on one unit, here over the device's own CDEF output of the case -- a Gram error that
    flips no tap downstream fails here."""
    import pipeline_cases as pc
    import pipeline_run as prun
    c, g = pc.CASES[case], pc.load(case)
    out = prun.run_gpu(case, ctx)
    L, hbd = svtgpu.lib(), c["bd"] > 8
    pad = [np.pad(np.ascontiguousarray(a, np.uint16 if hbd else np.uint8), 4, mode="edge") for a in out["cdef"]]
    srcs = [np.ascontiguousarray(a, np.uint16 if hbd else np.uint8) for a in out["src"]]
    Ms, Hs = [], []
    for row in g["wn_stats_meta"]:
        p, win, hs, he, vs, ve = (int(x) for x in row)
        d, s = pad[p], srcs[p]
        M, H = np.zeros(win * win, np.int64), np.zeros(win ** 4, np.int64)
        dp = _at(d, 4, 4, enc=hbd)
        sp = _at(s, 0, 0, enc=hbd)
        args = (win, dp, sp, hs, he, vs, ve, d.shape[1], s.shape[1], M.ctypes.data_as(ctypes.c_void_p),
                H.ctypes.data_as(ctypes.c_void_p))
        if hbd:
            L.svtgpu_av1_compute_stats_highbd(*args, c["bd"])
        else:
            L.svtgpu_av1_compute_stats(*args)
        Ms.append(M)
        Hs.append(H)
    M, H = np.concatenate(Ms), np.concatenate(Hs)
    if c["digest"]:
        assert pc.digest(M) == str(g["sha_wn_stats_M"]) and pc.digest(H) == str(g["sha_wn_stats_H"]), case
    else:
        np.testing.assert_array_equal(M, g["wn_stats_M"], err_msg=case)
        np.testing.assert_array_equal(H, g["wn_stats_H"], err_msg=case)


def test_lr_search_serial_measurement_mode_same_records(ctx):
    """svtgpu_lr_profile bit 7 (the roofline's isolated measurement: both LR chains on the caller's stream) changes
    only where the Wiener chain runs, never a result: records, frame types and picked units equal the default search."""
    w, h, bd, usize = 640, 360, 10, 64
    src, rec = _crop_pair(w, h, bd, seed=0x5EED0900)
    ctrls = oracle.lr_controls(1, 1, rdmult=7000, switchable=(300, 700, 900), wiener=(250, 800), sgrproj=(250, 900))
    unit_size = [usize, usize >> 1, usize >> 1]
    _, _, ft0, recs0 = _gpu_search(ctx, rec, src, bd, unit_size, ctrls)
    R, S = svtgpu.Frame(ctx, w, h, bd), svtgpu.Frame(ctx, w, h, bd)
    R.upload(rec)
    S.upload(src)
    st = svtgpu.LrState(ctx, w, h, unit_size)
    st.profile(True, events=True, serial=True)
    ft1, recs1 = st.search(R, S, ctrls, records=True)
    prof = st.profile(False)
    assert prof["searches"] == 1 and prof["projection"]["launches"] > 0 and prof["projection"]["ms_events"] > 0
    assert ft1 == ft0
    for p in range(3):
        np.testing.assert_array_equal(recs1[p], recs0[p])


@pytest.mark.parametrize("case", [1, 4, 10, 13])
def test_lr_search_async_equals_sync(ctx, case):
    """svtgpu_lr_search_frame_async + svtgpu_lr_apply_frame(frame_type = NULL) -- the search, the device RD finish and
    the apply in stream order with no host wait -- writes the same restored frame as the synchronous search + apply,
    and svtgpu_lr_read_result returns the reference's frame types."""
    c = list(lc.search_cases())[case]
    st, R, ft, recs = _gpu_search(ctx, c["rec"], c["src"], c["bd"], c["unit_size"], c["ctrls"])
    h, w = R.height, R.width
    D, O1, O2, S = (svtgpu.Frame(ctx, w, h, c["bd"]) for _ in range(4))
    D.upload(_coded(c["rec"], 3))
    S.upload(_coded(c["src"], 4))  # as _gpu_search
    st.apply(D, R, O1, ft)
    st2 = svtgpu.LrState(ctx, c["w"], c["h"], c["unit_size"])
    st2.search_async(R, S, c["ctrls"])
    st2.apply(D, R, O2, None)
    assert st2.read_result() == ft == c["ftype"]
    a, b = O1.download(), O2.download()
    for p in range(3):
        assert np.array_equal(a[p], b[p]), (c["name"], p)


FIN_WIN_CHILD = r"""
import sys
sys.path[:0] = [%r, %r, %r, %r]
import torch
if torch.cuda.is_available():
    torch.cuda.init()
import numpy as np
import svtgpu
import lr_cases as lc
import pipeline_run as prun
ctx = svtgpu.Context(0)
for c in lc.search_cases():
    h, w = c["rec"][0].shape
    pad = lambda planes, n: [np.pad(p, ((0, (-p.shape[0]) %% (8 if i == 0 else 4)),
                                        (0, (-p.shape[1]) %% (8 if i == 0 else 4))), mode="edge")
                             for i, p in enumerate(planes)]
    rec8, src8 = pad(c["rec"], 3), pad(c["src"], 4)
    R, S = (svtgpu.Frame(ctx, rec8[0].shape[1], rec8[0].shape[0], c["bd"]) for _ in range(2))
    R.upload(rec8), S.upload(src8)
    st = svtgpu.LrState(ctx, w, h, c["unit_size"])
    ft, recs = st.search(R, S, c["ctrls"], records=True)
    lc.compare_search(ft, c["units"], recs, c)
for case in %r:
    prun.check(case, prun.run_gpu(case, ctx, async_=True), "fin window")
print("ok")
"""


@pytest.mark.timeout(600)
def test_lr_finish_walk_evaluates_far_references():
    """The device RD finish's walks read a unit's decision / coefficient bits from the tables for references up to 63
    units back and evaluate the others at the step.  With the window cut to one unit (SVTGPU_LR_FIN_WIN=1, in a child
    process: the switch is read once) nearly every step takes the evaluation path; the reference's records, frame types
    and restored planes must not change (every LR golden case, the 1080p 8-bit and 4K 10-bit pipeline goldens)."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = FIN_WIN_CHILD % (root, os.path.join(root, "svt-av1_pro-anchor-v2.1.0-_amd"), os.path.join(root, "oracle"),
                            os.path.join(root, "tests"), ("mini10", "c1_1080p8", "c3_4k10"))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=550,
                       env=dict(os.environ, SVTGPU_LR_FIN_WIN="1"))
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stderr[-3000:]
