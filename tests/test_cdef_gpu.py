"""CDEF parity on the MI355X: HIP path (through the C ABI) vs golden vectors and vs the CPU oracle.

Bit-exact everywhere (integer pixel kernels; the luma distortion's double-precision formula is
evaluated with the reference's operation order and no FMA contraction)."""
import ctypes

import numpy as np
import pytest

import cdef_cases as cc
import oracle
import svtgpu
import synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    return svtgpu.Context(0)


# ------------------------------------------------------------------ per-block RTCD shims vs golden
def test_find_dir_shim_golden(ctx):
    L = svtgpu.lib()
    g = cc.load("cdef_find_dir.bin")
    for n in range(len(g["dir"])):
        img = np.ascontiguousarray(g["img"][n])
        var = ctypes.c_int32()
        d = L.svtgpu_cdef_find_dir(ctypes.c_void_p(img.ctypes.data), 8, ctypes.byref(var), int(g["bd"][n]) - 8)
        assert (d, var.value) == (g["dir"][n], g["var"][n]), n
    # dual form
    a, b = np.ascontiguousarray(g["img"][1]), np.ascontiguousarray(g["img"][4])
    v1, v2, d1, d2 = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_uint8(), ctypes.c_uint8()
    L.svtgpu_cdef_find_dir_dual(ctypes.c_void_p(a.ctypes.data), ctypes.c_void_p(b.ctypes.data), 8, ctypes.byref(v1),
                                ctypes.byref(v2), 2, ctypes.byref(d1), ctypes.byref(d2))
    assert (d1.value, v1.value, d2.value, v2.value) == (g["dir"][1], g["var"][1], g["dir"][4], g["var"][4])


def test_filter_block_shim_golden(ctx):
    L = svtgpu.lib()
    g = cc.load("cdef_filter_block.bin")
    bad = [n for n in range(len(g["out"]))
           if not np.array_equal(cc.run_filter_block(L.svtgpu_cdef_filter_block, g, n), g["out"][n])]
    assert not bad, bad[:10]


def test_cdef_dist_shim_golden(ctx):
    L = svtgpu.lib()
    g = cc.load("cdef_dist.bin")
    for n in range(len(g["dist"])):
        r = cc.run_cdef_dist(L.svtgpu_compute_cdef_dist_16bit, L.svtgpu_compute_cdef_dist_8bit, g, n)
        assert r == int(g["dist"][n]), n


def test_search_one_dual_shim_golden(ctx):
    L = svtgpu.lib()
    g = cc.load("cdef_search_one_dual.bin")
    for n in range(len(g["best"])):
        best, l0, l1, _ = cc.run_search_one_dual(L.svtgpu_search_one_dual, g, n)
        assert best == int(g["best"][n]), n
        assert l0 == list(g["lev_out"][n][0]) and l1 == list(g["lev_out"][n][1]), n


# ------------------------------------------------------------------ frame level vs oracle
FRAME_CASES = [
    # (width, height, bit_depth, cdef_level, p_skip, base_q_idx)
    (256, 192, 8, 1, 0.0, 128),
    (256, 192, 10, 1, 0.0, 128),
    (200, 136, 10, 1, 0.3, 200),   # partial FBs at right/bottom, skipped blocks
    (320, 120, 8, 2, 0.2, 60),     # chroma second pass untested (-1 → default_mse_uv)
    (192, 200, 10, 9, 0.1, 255),   # luma row subsampling 4, zero-fs bias off
    (136, 264, 8, 12, 0.5, 100),   # zero_fs_cost_bias 62
    (128, 128, 10, 5, 1.0, 90),    # every block skipped
]


def _gpu_pipeline(ctx, src, rec, bd, ctrls, q, mask, lam):
    h, w = rec[0].shape
    R = svtgpu.Frame(ctx, w, h, bd)
    S = svtgpu.Frame(ctx, w, h, bd)
    O = svtgpu.Frame(ctx, w, h, bd)
    R.upload(rec)
    S.upload(src)
    st = svtgpu.CdefState(ctx, w, h)
    st.set_block_mask(mask)
    st.search(R, S, ctrls, q)
    mse, skip, d, v = st.read()
    prm, fbs = st.pick(ctrls, q, lam)
    st.apply(R, O, prm)
    out = O.download()
    return (mse, skip, d, v), (prm, fbs), out


@pytest.mark.parametrize("case", FRAME_CASES, ids=lambda c: "x".join(map(str, c)))
def test_cdef_frame_pipeline_vs_oracle(ctx, case):
    w, h, bd, level, p_skip, q = case
    src, rec = synth.frame_pair(w, h, bd, seed=0x5EED0100 + w + h + bd)
    mask = synth.block_mask(w, h, seed=w * h, p_skip=p_skip)
    ctrls = svtgpu.cdef_controls(level)
    lam = 12345 + 77 * q
    (mse, skip, d, v), (prm, fbs), out = _gpu_pipeline(ctx, src, rec, bd, ctrls, q, mask, lam)
    omse, oskip, od, ov = oracle.cdef_search_frame(rec, src, bd, ctrls, q, mask)
    np.testing.assert_array_equal(skip, oskip)
    live = oskip == 0
    np.testing.assert_array_equal(mse[:, live], omse[:, live])
    # dir/var are only meaningful for listed blocks of searched FBs
    lm = np.zeros_like(od, dtype=bool)
    nhfb = (w // 4 + 15) // 16
    for fb in np.nonzero(live)[0]:
        fbr, fbc = divmod(fb, nhfb)
        for b in range(64):
            r, c = 8 * fbr + b // 8, 8 * fbc + b % 8
            lm[fb, b] = r < mask.shape[0] and c < mask.shape[1] and mask[r, c]
    np.testing.assert_array_equal(d[lm], od[lm])
    np.testing.assert_array_equal(v[lm], ov[lm])
    oprm, ofbs = oracle.cdef_pick(w, h, omse, oskip, ctrls, q, lam)
    assert prm.as_tuple() == oprm.as_tuple()
    np.testing.assert_array_equal(fbs, ofbs)
    oout = oracle.cdef_apply_frame(rec, bd, mask, od, ov, oprm, ofbs)
    for p in range(3):
        np.testing.assert_array_equal(out[p], oout[p], err_msg="plane %d" % p)


def test_cdef_1080p_8bit_config2_bit_exact(ctx):
    """BASELINE config 2: 1080p 8-bit CDEF search + apply, bit-exact vs the reference C semantics."""
    w, h, bd, q = 1920, 1080, 8, 128
    src, rec = synth.frame_pair(w, h, bd, seed=0x5EED0002)
    ctrls = svtgpu.cdef_controls(1)
    lam = 60000
    (mse, skip, d, v), (prm, fbs), out = _gpu_pipeline(ctx, src, rec, bd, ctrls, q, None, lam)
    omse, oskip, od, ov = oracle.cdef_search_frame(rec, src, bd, ctrls, q, None)
    np.testing.assert_array_equal(mse, omse)
    np.testing.assert_array_equal(d, od)
    np.testing.assert_array_equal(v, ov)
    oprm, ofbs = oracle.cdef_pick(w, h, omse, oskip, ctrls, q, lam)
    assert prm.as_tuple() == oprm.as_tuple()
    np.testing.assert_array_equal(fbs, ofbs)
    oout = oracle.cdef_apply_frame(rec, bd, None, od, ov, oprm, ofbs)
    for p in range(3):
        np.testing.assert_array_equal(out[p], oout[p])


def test_cdef_4k_10bit_properties(ctx):
    """Full-size config-3 CDEF: size-independent properties (the oracle is too slow at 4K)."""
    w, h, bd, q = 3840, 2160, 10, 128
    src, rec = synth.frame_pair(w, h, bd, seed=0x5EED0003)
    ctrls = svtgpu.cdef_controls(1)
    R, S, O = (svtgpu.Frame(ctx, w, h, bd) for _ in range(3))
    R.upload(rec)
    S.upload(src)
    st = svtgpu.CdefState(ctx, w, h)
    st.search(R, S, ctrls, q)
    mse1, skip, d, v = st.read()
    st.search(R, S, ctrls, q)  # deterministic
    mse2, _, _, _ = st.read()
    np.testing.assert_array_equal(mse1, mse2)
    assert not skip.any()
    # strength 0 (gi 0) is the unfiltered copy: its luma distortion equals the oracle's on that FB
    # spot-check a handful of FBs against the oracle on cropped 64x64-aligned windows
    nhfb = w // 64
    for fb in (0, nhfb - 1, 17 * nhfb + 29, len(skip) - 1):
        fbr, fbc = divmod(fb, nhfb)
        r0, c0 = 64 * max(fbr - 1, 0), 64 * max(fbc - 1, 0)
        r1, c1 = min(h, 64 * (fbr + 2)), min(w, 64 * (fbc + 2))
        crop = lambda planes: [planes[0][r0:r1, c0:c1]] + [p[r0 // 2:r1 // 2, c0 // 2:c1 // 2] for p in planes[1:]]
        # interior FBs of the crop see the same neighbourhood as in the full frame only if the crop
        # does not cut their +-3 px context: FB (fbr, fbc) sits fully inside with >= 64 px margin
        # except at real frame edges, which coincide with crop edges.
        om, _, _, _ = oracle.cdef_search_frame(crop(rec), crop(src), bd, ctrls, q, None)
        cw = c1 - c0
        lfb = (fbr - r0 // 64) * ((cw // 4 + 15) // 16) + (fbc - c0 // 64)
        np.testing.assert_array_equal(mse1[:, fb], om[:, lfb])
    prm, fbs = st.pick(ctrls, q, 60000)
    # zero strengths everywhere => apply is the identity
    zero = svtgpu.CdefParams()
    zero.cdef_damping = prm.cdef_damping
    st.apply(R, O, zero)
    for a, b in zip(O.download(), rec):
        np.testing.assert_array_equal(a, b)
    st.apply(R, O, prm)
    out = O.download()
    # filtered output stays within the sample range and differs from the input somewhere
    assert max(int(p.max()) for p in out) <= 1023
    assert any((a != b).any() for a, b in zip(out, rec))


@pytest.mark.parametrize("nb", [2, 3])
def test_cdef_band_search_allreduce(ctx, nb):
    """The multi-GPU split of bench.py on one device: each band's search into zeroed tables, the tables summed
    (what the RCCL all-reduce does), then the pick and a whole-frame apply == the one-band pipeline."""
    import torch
    w, h, bd, q, lam = 512, 328, 10, 128, 60000
    src, rec = synth.frame_pair(w, h, bd, seed=0x5EED0B00 + nb)
    R, S, O1, O2 = (svtgpu.Frame(ctx, w, h, bd) for _ in range(4))
    R.upload(rec)
    S.upload(src)
    ctrls = svtgpu.cdef_controls(1)
    full = svtgpu.CdefState(ctx, w, h)
    full.search(R, S, ctrls, q)
    prm1, fbs1 = full.pick(ctrls, q, lam)
    full.apply(R, O1, prm1)
    st = svtgpu.CdefState(ctx, w, h)
    nvfb = (h // 4 + 15) // 16
    tabs = [torch.zeros((2, st.nfb, 64), dtype=torch.int64, device="cuda"),
            torch.zeros(st.nfb, dtype=torch.uint8, device="cuda"),
            torch.zeros((st.nfb, 64), dtype=torch.uint8, device="cuda"),
            torch.zeros((st.nfb, 64), dtype=torch.int32, device="cuda")]
    total = [torch.zeros_like(t) for t in tabs]
    st.bind_tables(tabs[0].data_ptr(), tabs[1].data_ptr())
    st.bind_dir_tables(tabs[2].data_ptr(), tabs[3].data_ptr())
    for r in range(nb):
        st.set_fb_rows(*svtgpu.band(nvfb, nb, r))
        st.clear_tables()
        st.search(R, S, ctrls, q)
        torch.cuda.synchronize()
        for a, b in zip(total, tabs):
            a += b
    for a, b in zip(tabs, total):
        a.copy_(b)
    torch.cuda.synchronize()
    st.set_fb_rows(0, nvfb)
    prm2, fbs2 = st.pick(ctrls, q, lam)
    st.apply(R, O2, prm2)
    assert prm1.as_tuple() == prm2.as_tuple() and np.array_equal(fbs1, fbs2)
    for a, b in zip(O1.download(), O2.download()):
        assert np.array_equal(a, b)


@pytest.mark.parametrize("persist", ["1", "0"])
@pytest.mark.parametrize("top", [1 << 31, 1 << 40])
@pytest.mark.parametrize("w,h", [(1024, 512), (3840, 2160)])
def test_cdef_pick_bound_tables_vs_oracle(ctx, top, w, h, persist, monkeypatch):
    """The frame pick over arbitrary mse tables: entries just below 2^31 (the 32-bit accumulation path, sums of
    two entries up to 2^32 - 2) and up to 2^40 (the 64-bit path), random skipped FBs; bit-exact vs the oracle.
    Both pick paths: the persistent kernel (default; 3840x2160 fills its 64 chunks of 32 FBs) and the launch per
    step (SVTGPU_PICK_PERSIST=0; at 3840x2160 the default launch shape stages the largest FB chunks)."""
    import torch
    monkeypatch.setenv("SVTGPU_PICK_PERSIST", persist)
    q, lam = 128, 60000
    ctrls = svtgpu.cdef_controls(1)
    st = svtgpu.CdefState(ctx, w, h)
    rng = np.random.default_rng(top % 1000003)
    mse = (top - 1 - rng.integers(0, top // 64, size=(2, st.nfb, 64), dtype=np.int64)).astype(np.uint64)
    mse[:, :, 0] = rng.integers(0, top // 2, size=(2, st.nfb)).astype(np.uint64)  # strength 0 often best
    skip = (rng.random(st.nfb) < 0.1).astype(np.uint8)
    mse_t = torch.from_numpy(mse.view(np.int64)).cuda()
    skip_t = torch.from_numpy(skip).cuda()
    st.bind_tables(mse_t.data_ptr(), skip_t.data_ptr())
    torch.cuda.synchronize()
    prm, fbs = st.pick(ctrls, q, lam)
    oprm, ofbs = oracle.cdef_pick(w, h, mse, skip, ctrls, q, lam)
    assert prm.as_tuple() == oprm.as_tuple()
    assert np.array_equal(fbs, ofbs)
    # again on the same state (the persistent kernel's exchange words of the previous pick stay behind), then at a
    # level with fewer strengths (the words are cleared), then back
    for lv in (1, 5, 1):
        c2 = svtgpu.cdef_controls(lv)
        prm2, fbs2 = st.pick(c2, q, lam)
        oprm2, ofbs2 = oracle.cdef_pick(w, h, mse, skip, c2, q, lam)
        assert prm2.as_tuple() == oprm2.as_tuple() and np.array_equal(fbs2, ofbs2), lv


@pytest.mark.parametrize("persist", ["1", "0"])
@pytest.mark.parametrize("frac", [1.0, 0.999])
def test_cdef_pick_all_or_almost_all_skipped(ctx, frac, persist, monkeypatch):
    """Edge cases of the pick's compaction: every FB skipped (no rows: the chains return the reference's (1 << 63)
    sentinel and the RD choice keeps one zero strength) and a single live FB; both pick paths; bit-exact vs the
    oracle, skipped FBs get index 0."""
    import torch
    monkeypatch.setenv("SVTGPU_PICK_PERSIST", persist)
    w, h, q, lam = 1920, 1080, 128, 60000
    ctrls = svtgpu.cdef_controls(1)
    st = svtgpu.CdefState(ctx, w, h)
    rng = np.random.default_rng(1234)
    mse = rng.integers(0, 1 << 30, size=(2, st.nfb, 64), dtype=np.int64).astype(np.uint64)
    skip = np.ones(st.nfb, np.uint8)
    if frac < 1.0:
        skip[st.nfb // 2] = 0
    mse_t = torch.from_numpy(mse.view(np.int64)).cuda()
    skip_t = torch.from_numpy(skip).cuda()
    st.bind_tables(mse_t.data_ptr(), skip_t.data_ptr())
    torch.cuda.synchronize()
    prm, fbs = st.pick(ctrls, q, lam)
    oprm, ofbs = oracle.cdef_pick(w, h, mse, skip, ctrls, q, lam)
    assert prm.as_tuple() == oprm.as_tuple()
    assert np.array_equal(fbs, ofbs)


def _settle_calls(mse, skip, end=64):
    """First call of each greedy chain (nb = 1, 2, 4, 8; EbEncCdef.c:697-727) whose ordered selection repeats the
    one nb calls earlier -- from there on the device copies the chain's calls instead of recomputing them (the
    period shortcut in sod_step_kernel); None if the chain never settles.  numpy, for the coverage bookkeeping of
    the test below only."""
    keep = skip == 0
    m0 = mse[0][keep][:, :end].astype(np.int64)
    m1 = mse[1][keep][:, :end].astype(np.int64)
    V = m0[:, :, None] + m1[:, None, :]
    out = []
    for c in range(4):
        nb, sl, lev, res, first = 1 << c, [0] * 32, [], None, None
        for s in range(5 * nb + 1):
            if s > 0:
                prev = min(s - 1, nb - 1)
                sl[prev], sl[16 + prev] = res
                if nb <= s < 5 * nb:
                    sl[:nb - 1], sl[16:16 + nb - 1] = sl[1:nb], sl[17:16 + nb]
            lev.append(list(sl))
            if s == 5 * nb:
                break
            nsel = min(s, nb - 1)
            if first is None and s - nb >= nb and all(lev[s][q] == lev[s - nb][q] and lev[s][16 + q] == lev[s - nb][16 + q]
                                                      for q in range(nb - 1)):
                first = s
            b = (np.full(m0.shape[0], 1 << 62, np.int64) if nsel == 0 else
                 np.min(np.stack([m0[:, sl[q]] + m1[:, sl[16 + q]] for q in range(nsel)]), axis=0))
            e = int(np.argmin(np.minimum(V, b[:, None, None]).sum(0)))
            res = (e // end, e % end)
        out.append(first)
    return out


@pytest.mark.parametrize("scale_hi", [1 << 20, 1 << 14])
def test_cdef_pick_settled_chains_vs_oracle(ctx, monkeypatch, scale_hi):
    """The launch-per-step pick's period shortcut: convex per-FB strength curves (random optimum and scale per FB)
    whose greedy chains settle at different calls -- and, for some seeds, never -- bit-exact vs the oracle, the
    pick repeated on the same state (the step values of the previous pick stay behind).  scale_hi 2^20: entries above
    2^31 (the 64-bit path); 2^14: every entry below 2^31 (pick_gather's `wide` stays 0), so the steps stage the low words in LDS (the padded
    132-dword rows, the 32-bit per-FB best) -- both with settled and unsettled chains."""
    import torch
    monkeypatch.setenv("SVTGPU_PICK_PERSIST", "0")
    w, h, q, lam = 1920, 1080, 128, 60000
    ctrls = svtgpu.cdef_controls(1)
    st = svtgpu.CdefState(ctx, w, h)
    seen = set()
    for seed in range(6):
        rng = np.random.default_rng(seed)
        j = np.arange(64)
        opt = rng.integers(0, 64, size=(2, st.nfb, 1))
        scale = rng.integers(1 << 10, scale_hi, size=(2, st.nfb, 1))
        mse = (scale * (64 + (j - opt) ** 2) + rng.integers(0, 1 << 12, size=(2, st.nfb, 64))).astype(np.uint64)
        assert (mse.max() < (1 << 31)) == (scale_hi < (1 << 17))
        skip = (rng.random(st.nfb) < 0.1).astype(np.uint8)
        seen.update(x is None for x in _settle_calls(mse, skip)[1:])
        mse_t = torch.from_numpy(mse.view(np.int64)).cuda()
        skip_t = torch.from_numpy(skip).cuda()
        st.bind_tables(mse_t.data_ptr(), skip_t.data_ptr())
        torch.cuda.synchronize()
        oprm, ofbs = oracle.cdef_pick(w, h, mse, skip, ctrls, q, lam)
        for _ in range(2):
            prm, fbs = st.pick(ctrls, q, lam)
            assert prm.as_tuple() == oprm.as_tuple() and np.array_equal(fbs, ofbs), seed
    assert seen == {True, False}  # settled and unsettled chains both covered


@pytest.mark.parametrize("persist,fallback", [("0", "persist"), ("0", "steps"), ("1", "persist")])
def test_cdef_pick_async_vs_oracle(ctx, monkeypatch, persist, fallback):
    """svtgpu_cdef_pick_async (no host wait: the settle check's outcome reaches the later steps through a device flag,
    the parameters stay on the device) on the settled / unsettled tables of the test above: svtgpu_cdef_read_params
    equals the oracle's pick on every seed, three picks in a row on one state (the checkpoint T then moves from the
    records the earlier picks left, read without a wait), and the apply from device parameters writes the same planes
    as the apply with the host parameters.  After the check the asynchronous pick launches either one persistent
    launch that recomputes the pick when a chain has not settled (default) or the remaining steps, each returning at
    once when every chain has (SVTGPU_PICK_ASYNC_FALLBACK=steps); the unsettled seeds exercise both."""
    import torch
    monkeypatch.setenv("SVTGPU_PICK_PERSIST", persist)
    monkeypatch.setenv("SVTGPU_PICK_ASYNC_FALLBACK", fallback)
    w, h, q, lam = 1920, 1080, 128, 60000
    ctrls = svtgpu.cdef_controls(1)
    st = svtgpu.CdefState(ctx, w, h)
    seen = set()
    for seed in range(6):
        rng = np.random.default_rng(seed)
        j = np.arange(64)
        opt = rng.integers(0, 64, size=(2, st.nfb, 1))
        scale = rng.integers(1 << 10, 1 << 14, size=(2, st.nfb, 1))
        mse = (scale * (64 + (j - opt) ** 2) + rng.integers(0, 1 << 12, size=(2, st.nfb, 64))).astype(np.uint64)
        skip = (rng.random(st.nfb) < 0.1).astype(np.uint8)
        seen.update(x is None for x in _settle_calls(mse, skip)[1:])
        mse_t = torch.from_numpy(mse.view(np.int64)).cuda()
        skip_t = torch.from_numpy(skip).cuda()
        st.bind_tables(mse_t.data_ptr(), skip_t.data_ptr())
        torch.cuda.synchronize()
        oprm, ofbs = oracle.cdef_pick(w, h, mse, skip, ctrls, q, lam)
        for _ in range(3):
            st.pick_async(ctrls, q, lam)
            prm, fbs = st.read_params()
            assert prm.as_tuple() == oprm.as_tuple() and np.array_equal(fbs, ofbs), seed
    assert seen == {True, False}
    # the apply from device parameters: a real frame, search + async pick + apply(None) vs the synchronous pick
    w2, h2 = 640, 384
    src, rec = synth.frame_pair(w2, h2, 10, seed=0x5EED0177)
    S, R, O1, O2 = (svtgpu.Frame(ctx, w2, h2, 10) for _ in range(4))
    S.upload(src), R.upload(rec)
    st2 = svtgpu.CdefState(ctx, w2, h2)
    st2.search(R, S, ctrls, q)
    prm1, fbs1 = st2.pick(ctrls, q, lam)
    st2.apply(R, O1, prm1)
    st2.pick_async(ctrls, q, lam)
    st2.apply(R, O2, None)
    prm2, fbs2 = st2.read_params()
    assert prm1.as_tuple() == prm2.as_tuple() and np.array_equal(fbs1, fbs2)
    for a, b in zip(O1.download(), O2.download()):
        assert np.array_equal(a, b)
