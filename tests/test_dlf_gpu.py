"""Deblocking parity on the MI355X: HIP path (through the C ABI) vs the reference's golden vectors
and vs the CPU oracle.  Bit-exact (integer pixel filters; the level search compares integer SSEs)."""
import ctypes

import numpy as np
import pytest

import cdef_cases as cc
import dlf_cases as dc
import oracle
import svtgpu
import synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    return svtgpu.Context(0)


def _gpu_filter(ctx, planes, bd, mi, params, ps=0, pe=3, crop=None):
    h, w = planes[0].shape
    f = svtgpu.Frame(ctx, w, h, bd)
    f.upload(planes)
    st = svtgpu.DlfState(ctx, w, h)
    if crop and crop != (w, h):
        st.set_crop(*crop)
    st.set_mode_info(mi)
    st.filter(f, params, ps, pe)
    return f.download()


# ------------------------------------------------------------------ per-segment RTCD shims vs golden
def test_lpf_shims_golden(ctx):
    L = svtgpu.lib()
    g = cc.load("dlf_lpf.bin")
    meta, inp, out = g["meta"], g["in"], g["out"]
    bad = []
    for n in range(len(meta)):
        kind, fn, bl, li, th = (int(x) for x in meta[n])
        vertical, length = fn >= 4, (4, 6, 8, 14)[fn & 3]
        lowbd = kind == 8
        win = np.zeros((16, 16), np.uint8 if lowbd else np.uint16)
        for i in range(4):
            if vertical:
                win[8 + i, :] = inp[n][i]
            else:
                win[:, 8 + i] = inp[n][i]
        thr = [np.full(16, v, np.uint8) for v in (bl, li, th)]
        base = ctypes.c_void_p(win.ctypes.data + (8 * 16 + 8) * win.itemsize)
        name = "svtgpu_%slpf_%s" % ("" if lowbd else "highbd_", dc.LPF_NAMES[fn])
        args = [base, 16] + [ctypes.c_void_p(t.ctypes.data) for t in thr]
        getattr(L, name)(*(args if lowbd else args + [8 if kind == 108 else kind]))
        got = np.stack([win[8 + i, :] if vertical else win[:, 8 + i] for i in range(4)]).astype(np.uint16)
        if not np.array_equal(got, out[n]):
            bad.append((n, name))
    assert not bad, bad[:10]


# ------------------------------------------------------------------ frame filter vs reference golden
@pytest.mark.parametrize("case", list(range(11)))
def test_dlf_frame_golden(ctx, case):
    """The reference's svt_av1_loop_filter_frame (gen_golden_dlf.c); cases 8-10 on pictures off the 8-sample grid
    (svtgpu_dlf_set_crop: no edge at or past the unpadded size is filtered)."""
    c = list(dc.frame_cases())[case]
    got = _gpu_filter(ctx, c["inp"], c["bd"], c["mi"], c["params"], c["plane_start"], c["plane_end"], c["crop"])
    for p in range(3):
        assert np.array_equal(got[p], c["out"][p]), (c["name"], p)


# ------------------------------------------------------------------ frame filter vs oracle
FRAME_CASES = [
    # w, h, bd, seed, params kwargs, mi kwargs
    (640, 360, 10, 1, dict(fl0=32, fl1=16, flu=16, flv=12), {}),
    (392, 216, 8, 2, dict(fl0=63, fl1=63, flu=40, flv=63, sharpness=3), dict(segments=True)),
    (520, 264, 10, 3, dict(fl0=20, fl1=44, flu=8, flv=0, ref_deltas=(1, 0, 0, 0, -1, 0, -1, -1),
                           mode_deltas=(0, 0)), dict(p_skip=0.8)),
    (256, 256, 8, 4, dict(fl0=9, fl1=30, flu=30, flv=9, sharpness=7, ref_deltas=(3, -2, 5, 0, -7, 1, 2, -1),
                          mode_deltas=(4, -3)), dict(p_intra=0.7, segments=True, sb=128)),
]


def _params(kw, seed):
    kw = dict(kw)
    seg = kw.pop("segments", False)
    if seg:
        r = np.random.default_rng(seed)
        kw["seg_enabled"] = r.integers(0, 2, (8, 8))
        kw["seg_data"] = r.integers(-63, 64, (8, 8))
    return svtgpu.LfParams.make(kw.pop("fl0"), kw.pop("fl1"), kw.pop("flu"), kw.pop("flv"), **kw)


@pytest.mark.parametrize("w,h,bd,seed,pk,mk", FRAME_CASES)
def test_dlf_frame_vs_oracle(ctx, w, h, bd, seed, pk, mk):
    src, rec = synth.frame_pair(w, h, bd, seed=0x5EED0100 + seed)
    mi = dc.random_mode_info(w, h, seed, **mk)
    prm = _params(dict(pk, segments=mk.get("segments", False)), seed)
    want = oracle.dlf_frame(rec, bd, mi, prm)
    got = _gpu_filter(ctx, rec, bd, mi, prm)
    for p in range(3):
        assert np.array_equal(got[p], want[p]), p
    assert any(not np.array_equal(want[p], rec[p]) for p in range(3))
    # out-of-place form
    A, B = svtgpu.Frame(ctx, w, h, bd), svtgpu.Frame(ctx, w, h, bd)
    A.upload(rec)
    st = svtgpu.DlfState(ctx, w, h)
    st.set_mode_info(mi)
    st.filter_to(A, B, prm)
    got2, back = B.download(), A.download()
    for p in range(3):
        assert np.array_equal(got2[p], want[p]) and np.array_equal(back[p], rec[p]), p


def test_dlf_frame_4k10_vs_oracle(ctx):
    w, h, bd = 3840, 2160, 10
    src, rec = synth.frame_pair(w, h, bd, seed=0x5EED0003)
    mi = synth.mode_info(w, h, 3)
    prm = svtgpu.LfParams.make(32, 16, 16, 16)
    want = oracle.dlf_frame(rec, bd, mi, prm)
    got = _gpu_filter(ctx, rec, bd, mi, prm)
    for p in range(3):
        assert np.array_equal(got[p], want[p]), p


# ------------------------------------------------------------------ level search vs oracle
PICK_CASES = [
    # w, h, bd, seed, start levels, dlf_avg, dlf_avg_uv, tl, early_exit, only4x4
    (320, 192, 10, 11, (20, 20, 8, 8), 0, 0, 0, 0, 0),   # dlf level 1 (EncModeConfig.c:1569-1576)
    (320, 192, 10, 15, (32, 32, 16, 16), 0, 0, 0, 2, 0),
    (256, 128, 8, 12, (0, 0, 0, 0), 0, 0, 0, 1, 0),
    (384, 200, 10, 13, (40, 36, 12, 30), 1, 1, 1, 2, 1),
    (192, 192, 8, 14, (63, 5, 63, 0), 0, 1, 0, 3, 0),
    (320, 256, 10, 16, (24, 24, 4, 50), 0, 0, 0, 0, 0),  # U and V searches of different lengths share launches
    (264, 136, 10, 17, (12, 40, 60, 2), 0, 0, 0, 0, 1),
]


@pytest.mark.parametrize("w,h,bd,seed,lv,avg,avg_uv,tl,ee,o4", PICK_CASES)
def test_dlf_pick_vs_oracle(ctx, w, h, bd, seed, lv, avg, avg_uv, tl, ee, o4):
    src, rec = synth.frame_pair(w, h, bd, seed=0x5EED0200 + seed)
    mi = dc.random_mode_info(w, h, seed, p_skip=0.3)
    prm = svtgpu.LfParams.make(*lv, ref_deltas=(1, 0, 0, 0, -1, 0, -1, -1), mode_deltas=(0, 0))
    want = oracle.dlf_pick(rec, src, bd, mi, prm, avg, avg_uv, tl, ee, o4)
    R, S = svtgpu.Frame(ctx, w, h, bd), svtgpu.Frame(ctx, w, h, bd)
    R.upload(rec)
    S.upload(src)
    st = svtgpu.DlfState(ctx, w, h)
    st.set_mode_info(mi)
    got = st.pick(R, S, prm, avg, avg_uv, tl, ee, o4)
    assert got.levels() == want.levels()
    # recon is left unfiltered by the search
    back = R.download()
    for p in range(3):
        assert np.array_equal(back[p], rec[p])


def test_plane_sse(ctx):
    for bd in (8, 10):
        src, rec = synth.frame_pair(200, 120, bd, seed=0x5EED0300 + bd)
        A, B = svtgpu.Frame(ctx, 200, 120, bd), svtgpu.Frame(ctx, 200, 120, bd)
        A.upload(src)
        B.upload(rec)
        for p in range(3):
            want = int(((src[p].astype(np.int64) - rec[p].astype(np.int64)) ** 2).sum())
            assert svtgpu.plane_sse(A, B, p) == want


# ------------------------------------------------------------------ mode info handed over in device memory
@pytest.mark.parametrize("w,h,bd,seed,pk,mk", FRAME_CASES[:3])
def test_dlf_mode_info_device_matches_host(ctx, w, h, bd, seed, pk, mk):
    """svtgpu_dlf_set_mode_info_device (the grid already in HBM, checked by the records kernel) filters and searches
    exactly like the host hand-over; a grid with a record out of range is reported by the next pick."""
    import torch
    src, rec = synth.frame_pair(w, h, bd, seed=0x5EED0100 + seed)
    mi = dc.random_mode_info(w, h, seed, **mk)
    prm = _params(dict(pk, segments=mk.get("segments", False)), seed)
    want = oracle.dlf_frame(rec, bd, mi, prm)
    R, S, O = (svtgpu.Frame(ctx, w, h, bd) for _ in range(3))
    R.upload(rec)
    S.upload(src)
    d_mi = torch.from_numpy(np.ascontiguousarray(mi).view(np.uint8).reshape(-1).copy()).cuda()
    host, dev = svtgpu.DlfState(ctx, w, h), svtgpu.DlfState(ctx, w, h)
    host.set_mode_info(mi)
    dev.set_mode_info_device(d_mi)
    dev.filter_to(R, O, prm)
    got = O.download()
    for p in range(3):
        assert np.array_equal(got[p], want[p]), p
    start = svtgpu.LfParams.make(16, 16, 8, 8)
    a = host.pick(R, S, start)
    b = dev.pick(R, S, start)
    assert a.levels() == b.levels()
    bad = np.ascontiguousarray(mi).copy()
    bad.view(np.uint8).reshape(-1, 8)[len(bad.reshape(-1)) // 2, 0] = 200  # bsize out of range
    dev.set_mode_info_device(torch.from_numpy(bad.view(np.uint8).reshape(-1).copy()).cuda())
    with pytest.raises(svtgpu.SvtGpuError, match="error"):
        dev.pick(R, S, start)
    dev.set_mode_info_device(d_mi)  # the flag was cleared when reported
    assert dev.pick(R, S, start).levels() == a.levels()
