"""Pins the CPU restatement (oracle/) to golden vectors produced by the reference's own C kernels
(oracle/ref_harness/gen_golden_cdef.c, built from /root/reference by oracle/ref.mk)."""
import numpy as np
import pytest

import cdef_cases as cc
import oracle


@pytest.fixture(scope="module")
def L():
    return oracle.lib()


def test_find_dir_golden(L):
    g = cc.load("cdef_find_dir.bin")
    import ctypes
    for n in range(len(g["dir"])):
        img = np.ascontiguousarray(g["img"][n])
        var = ctypes.c_int32()
        d = L.oracle_cdef_find_dir(ctypes.c_void_p(img.ctypes.data), 8, ctypes.byref(var), int(g["bd"][n]) - 8)
        assert d == g["dir"][n] and var.value == g["var"][n], n
    # every direction is exercised
    assert len(set(g["dir"].tolist())) == 8


def test_filter_block_golden(L):
    g = cc.load("cdef_filter_block.bin")
    bad = [n for n in range(len(g["out"]))
           if not np.array_equal(cc.run_filter_block(L.oracle_cdef_filter_block, g, n), g["out"][n])]
    assert not bad, bad[:10]


def test_cdef_dist_golden(L):
    g = cc.load("cdef_dist.bin")
    for n in range(len(g["dist"])):
        r = cc.run_cdef_dist(L.oracle_compute_cdef_dist_16bit, L.oracle_compute_cdef_dist_8bit, g, n)
        assert r == int(g["dist"][n]), n


def test_search_one_dual_golden(L):
    g = cc.load("cdef_search_one_dual.bin")
    for n in range(len(g["best"])):
        best, l0, l1, _ = cc.run_search_one_dual(L.oracle_search_one_dual, g, n)
        assert best == int(g["best"][n]), n
        assert l0 == list(g["lev_out"][n][0]) and l1 == list(g["lev_out"][n][1]), n


def test_controls_level1_match_encmodeconfig():
    c = oracle.controls(1)  # EncModeConfig.c:866-904
    assert c.first_pass_fs_num == 16 and c.default_second_pass_fs_num == 48
    assert list(c.default_first_pass_fs[:16]) == list(range(0, 64, 4))
    assert list(c.default_second_pass_fs[:48]) == [p + j for p in range(0, 64, 4) for j in (1, 2, 3)]
    assert c.subsampling_factor == 1 and c.zero_fs_cost_bias == 0
    c9 = oracle.controls(9)  # :1114-1133
    assert c9.first_pass_fs_num == 2 and list(c9.default_first_pass_fs[:2]) == [0, 60]
    assert list(c9.default_second_pass_fs[:2]) == [2, 62] and list(c9.default_second_pass_fs_uv[:2]) == [-1, -1]
    assert c9.subsampling_factor == 4
    with pytest.raises(ValueError):
        oracle.controls(0)  # CDEF off
    for lvl in (11, 14, 15, 17):  # use_reference_cdef_fs levels (:1135-1300)
        assert oracle.controls(lvl).use_reference_cdef_fs == 1


# ---------------------------------------------------------------- deblocking (gen_golden_dlf.c)
def test_lpf_golden():
    import dlf_cases as dc
    g = cc.load("dlf_lpf.bin")
    meta, inp, out = g["meta"], g["in"], g["out"]
    bad = []
    for n in range(len(meta)):
        kind, fn, bl, li, th = (int(x) for x in meta[n])
        bd = 8 if kind == 108 else kind
        got = oracle.lpf_lines(inp[n], bd, fn, bl, li, th, lowbd=(kind == 8))
        if not np.array_equal(got, out[n]):
            bad.append((n, kind, dc.LPF_NAMES[fn]))
    assert not bad, bad[:10]
    # the sweep exercises the flat (6/8/14-tap) paths, not only filter4
    changed_far = sum(int(np.any(inp[n][:, [1, 2, 13, 14]] != out[n][:, [1, 2, 13, 14]])) for n in range(len(meta)))
    assert changed_far > 50


def test_dlf_frame_golden():
    import dlf_cases as dc
    n = 0
    for c in dc.frame_cases():
        got = oracle.dlf_frame(c["inp"], c["bd"], c["mi"], c["params"], c["plane_start"], c["plane_end"], c["crop"])
        for p in range(3):
            assert np.array_equal(got[p], c["out"][p]), (c["name"], p)
        n += 1
    assert n >= 11


# ---------------------------------------------------------------- MD distortion (gen_golden_md.c)
MD_SIZES = [(4, 4), (4, 8), (8, 4), (8, 8), (8, 16), (16, 8), (16, 16), (16, 32), (32, 16), (32, 32), (32, 64),
            (64, 32), (64, 64), (64, 128), (128, 64), (128, 128), (4, 16), (16, 4), (8, 32), (32, 8), (16, 64),
            (64, 16)]


def md_case(g, si, c):
    """(src16, ref16, src8, ref8) views of golden case c of size si (the 8-bit kernels saw the low byte;
    case 1 is the maximum-difference pattern 255/0)."""
    s16, r16 = g["s%d_src" % si][c], g["s%d_ref" % si][c]
    if c == 1:
        return s16, r16, np.full(s16.shape, 255, np.uint8), np.zeros(r16.shape, np.uint8)
    return s16, r16, (s16 & 255).astype(np.uint8), (r16 & 255).astype(np.uint8)


def test_md_dist_golden():
    L = oracle.lib()
    import ctypes
    g = cc.load("md_dist.bin")
    P = lambda a: ctypes.c_void_p(a.ctypes.data)
    for si, (w, h) in enumerate(MD_SIZES):
        res = g["s%d_res" % si]
        for c in range(res.shape[0]):
            s16, r16, s8, r8 = (np.ascontiguousarray(a) for a in md_case(g, si, c))
            st = s16.shape[1]
            sse = ctypes.c_uint32()
            assert L.oracle_sad(P(s8), st, P(r8), st, w, h) == res[c][0], (w, h, c)
            assert L.oracle_variance(P(s8), st, P(r8), st, w, h, ctypes.byref(sse)) == res[c][1], (w, h, c)
            assert sse.value == res[c][2]
            assert L.oracle_highbd_10_variance(P(s16), st, P(r16), st, w, h, ctypes.byref(sse)) == res[c][3], (w, h, c)
            assert sse.value == res[c][4]
            assert L.oracle_sad16(P(s16), st, P(r16), st, w, h) == res[c][5]
            for k, off in enumerate((0, 1, st, 3 * st + 2)):
                rr = np.ascontiguousarray(r8.reshape(-1)[off:])
                assert L.oracle_sad(P(s8), st, P(rr), st, w, h) == res[c][6 + k]
            assert L.oracle_sse(P(s8), st, P(r8), st, w, h) & 0xFFFFFFFF == res[c][10]
            assert (L.oracle_sse16(P(s16), st, P(r16), st, w, h) >> 4) & 0xFFFFFFFF == res[c][11]
    # known answers: zero difference -> 0, maximum difference -> var 0 with full sse
    assert g["s12_res"][0][0] == 0 and g["s12_res"][1][0] == 255 * 4096 and g["s12_res"][1][1] == 0


def test_md_batch_oracle_consistent():
    """The oracle batch = the pinned per-block kernels on the gathered (edge-clamped) blocks."""
    import md_cases as mc
    import synth
    w, h, bd, nref = 136, 72, 10, 2
    src, _ = synth.frame_pair(w, h, bd, seed=7)
    refs = mc.ref_frames(w, h, bd, nref, 7)
    mv = mc.mvs(w, h, nref, 7, rng_max=40)
    out = oracle.md_dist_batch(src[0], refs, bd, mv)
    rng = np.random.default_rng(0)
    offs = np.cumsum([0] + [4096 // (sw * sh) for sw, sh in oracle.MD_SHAPES])
    nsbx = (w + 63) // 64
    for _ in range(60):
        sb, r, s = rng.integers(0, out.shape[0]), rng.integers(0, nref), rng.integers(0, 19)
        sw, sh = oracle.MD_SHAPES[s]
        b = rng.integers(0, 4096 // (sw * sh))
        by, bx = (b // (64 // sw)) * sh, (b % (64 // sw)) * sw
        oy, ox = (sb // nsbx) * 64 + by, (sb % nsbx) * 64 + bx
        ys, xs = np.clip(np.arange(oy, oy + sh), 0, h - 1), np.clip(np.arange(ox, ox + sw), 0, w - 1)
        yr = np.clip(np.arange(oy, oy + sh) + mv[sb, r, 1], 0, h - 1)
        xr = np.clip(np.arange(ox, ox + sw) + mv[sb, r, 0], 0, w - 1)
        a, c = src[0][np.ix_(ys, xs)], refs[r][np.ix_(yr, xr)]
        want = oracle.block_dist(a, c, sw, sh, bd)
        k = offs[s] + b
        assert tuple(int(x) for x in out[sb, r, :, k]) == want


# ---------------------------------------------------------------- loop restoration (gen_golden_lr.c)
def test_wiener_golden():
    g = cc.load("lr_wiener.bin")
    for n in range(len(g["meta"])):
        bd, w, h = (int(x) for x in g["meta"][n])
        got = oracle.wiener_convolve(g["in%d" % n], w, h, g["taps"][n][:8], g["taps"][n][8:], bd)
        assert np.array_equal(got, g["out%d" % n]), (n, bd, w, h)


def test_sgr_golden():
    g = cc.load("lr_sgr.bin")
    eps_seen = set()
    for n in range(len(g["meta"])):
        bd, w, h, eps, x0, x1 = (int(x) for x in g["meta"][n])
        f0, f1 = oracle.sgr_filter(g["in%d" % n], w, h, eps, bd)
        if eps < 10 or eps >= 14:
            assert np.array_equal(f0, g["flt0_%d" % n]), (n, eps)
        if eps < 14:
            assert np.array_equal(f1, g["flt1_%d" % n]), (n, eps)
        assert np.array_equal(oracle.sgr_apply(g["in%d" % n], w, h, eps, (x0, x1), bd), g["out%d" % n]), (n, eps)
        eps_seen.add(eps)
    assert eps_seen == set(range(16))


def test_lr_frame_golden():
    import lr_cases as lc
    n = 0
    for c in lc.frame_cases():
        got = oracle.lr_apply_frame(c["dlf"], c["cdef"], c["bd"], c["frame_type"], c["unit_size"], c["units"])
        for p in range(3):
            assert np.array_equal(got[p], c["out"][p]), (c["name"], p)
        n += 1
    assert n >= 6


def test_lr_search_golden():
    import lr_cases as lc
    n = 0
    for c in lc.search_cases():
        ft, units, recs = oracle.lr_search_frame(c["rec"], c["src"], c["bd"], c["unit_size"], c["ctrls"])
        lc.compare_search(ft, units, recs, c)
        n += 1
    assert n >= 6


def test_compute_stats_golden():
    g = cc.load("lr_stats.bin")
    L = oracle.lib()
    for n in range(len(g["meta"])):
        bd, win, w, h, st, _ = (int(x) for x in g["meta"][n])
        d, s = g["dgd%d" % n].copy(), g["src%d" % n].copy()
        M, H = np.zeros(win * win, np.int64), np.zeros(win ** 4, np.int64)
        L.oracle_compute_stats(win, oracle.ptr(d), oracle.ptr(s), st, w, h, bd, oracle.ptr(M), oracle.ptr(H))
        assert np.array_equal(M, g["M%d" % n]) and np.array_equal(H, g["H%d" % n]), (n, bd, win)


# ---- open-loop ME SAD (me_oracle.c vs the reference's EbMotionEstimation.c / EbComputeSAD_C.c) ----
def test_oracle_me_search_vs_reference():
    import me_cases as mc
    for src, refs, origin, saw, sah, sub, sad, mv in mc.frames(mc.golden()):
        osad, omv = oracle.me_search(src, refs, origin, saw, sah, sub)
        np.testing.assert_array_equal(osad, sad)
        np.testing.assert_array_equal(omv, mv)


def test_oracle_sad_loop_vs_reference():
    import me_cases as mc
    for s, r, m in mc.loop_cases(mc.golden()):
        bw, bh, saw, sah, ss, rs, srr, skip, best, c = m
        got = oracle.sad_loop(s, ss, r, rs, bh, bw, srr, skip, saw, sah)
        want_c = ((c & 0xFFFF) ^ 0x8000) - 0x8000, ((c >> 16) ^ 0x8000) - 0x8000
        assert got[0] == best, m
        if best < 0xffffff:
            assert got[1:] == want_c, m


# ---- frame-buffer work (frame_oracle.c vs the reference's EbPackUnPack_C.c / EbMcp.c / EbRestoration.c) ----
def test_oracle_frame_ops_vs_reference():
    import frame_cases as fc
    g = fc.golden()
    for src, d0, d1, w, h, ss, ds in fc.conv_cases(g):
        d = d0.copy()
        oracle.convert(src, ss, d, ds, w, h)
        np.testing.assert_array_equal(d, d1)
    for b0, b1, w, h, st, pw, ph in fc.pad_cases(g):
        b = b0.copy()
        oracle.pad(b, st, w, h, pw, ph)
        np.testing.assert_array_equal(b, b1)
    for b0, b1, w, h, st, bh, bv, off in fc.ext_cases(g):
        b = b0.copy()
        oracle.extend(b, off, st, w, h, bh, bv)
        np.testing.assert_array_equal(b, b1)


def test_oracle_pme_sad_loop_vs_reference():
    import ctypes
    import me_cases as mc
    for p, keep, s, r, m in mc.pme_cases(mc.golden()):
        bw, bh, saw, sah, step, ss, rs = m[:7]
        best, bx, by = ctypes.c_uint32(m[10] & 0xFFFFFFFF), ctypes.c_int16(111), ctypes.c_int16(-111)
        oracle.lib().oracle_pme_sad_loop(ctypes.byref(p), oracle.ptr(s), ss, oracle.ptr(r), rs, bh, bw,
                                         ctypes.byref(best), ctypes.byref(bx), ctypes.byref(by), m[13], m[14], saw, sah,
                                         step, m[15], m[16])
        assert (best.value, bx.value, by.value) == (m[17] & 0xFFFFFFFF, m[18], m[19]), m


def test_oracle_md_batch_sb_range():
    """The SB-range oracle (used on 8K subsets) equals the matching rows of the whole-frame oracle."""
    import md_cases as mc
    import synth
    w, h, bd, nref = 200, 136, 10, 2
    src, _ = synth.frame_pair(w, h, bd, seed=0x5EED0590)
    refs = mc.ref_frames(w, h, bd, nref, 0x5EED0591)
    mv = mc.mvs(w, h, nref, 3, rng_max=30)
    whole = oracle.md_dist_batch(src[0], refs, bd, mv)
    for b, e in ((0, 3), (5, 12), (9, 12)):
        assert np.array_equal(oracle.md_dist_batch(src[0], refs, bd, mv, sb_range=(b, e)), whole[b:e])


# ---- CCSO (ccso_oracle.c vs the fork's EbCcso.c / EbPickccso.c, tests/golden/ccso.bin) ----
def test_oracle_ccso_extend_vs_reference():
    import ccso_cases as xc
    cases = [c for c in xc.search_cases(xc.golden()) if c["ext"] is not None]
    assert cases
    for c in cases:
        np.testing.assert_array_equal(oracle.ccso_extend(c["pre"]), c["ext"], err_msg="case %d" % c["n"])


def test_oracle_ccso_apply_vs_reference():
    """ccso_frame with random ccso_info and block flags (every filter support, band-offset-only, 1-128 bands)."""
    import ccso_cases as xc
    for c in xc.apply_cases(xc.golden()):
        ext = oracle.ccso_extend(c["pre"])
        for p in range(3):
            got = oracle.ccso_apply_plane(ext, 8, p, c["inp"][p], c["params"][p], c["flags"][p])
            np.testing.assert_array_equal(got, c["out"][p], err_msg="case %d plane %d" % (c["n"], p))


def test_oracle_ccso_search_vs_reference():
    """ccso_search (every plane's derive_ccso_filter) and, at 8 bits, ccso_frame applying its result: the frame header
    fields, the LUT, the block flags and the filtered planes equal the reference's; the cases include planes that
    stay off (no coding-error bias at a high rdmult) and the rdmult overflow that returns before any search."""
    import ccso_cases as xc
    cases = xc.search_cases(xc.golden())
    assert any(c["params"][0].enable for c in cases) and any(not c["params"][0].enable for c in cases)
    for c in cases:
        ext = oracle.ccso_extend(c["pre"])
        rc, prms, flags, ff = oracle.ccso_search_frame(ext, c["org"], c["rec"], c["bd"], c["rdmult"], c["q"])
        msg = "case %d (%dx%d %d-bit)" % (c["n"], c["w"], c["h"], c["bd"])
        assert ff == c["frame_flag"], msg
        for p in range(3):
            want = c["params"][p]
            if rc == 1:  # nothing searched: the header keeps its (zeroed) fields
                assert not want.enable, msg
                continue
            assert prms[p].fields() == want.fields(), "%s plane %d" % (msg, p)
            if want.enable:
                np.testing.assert_array_equal(prms[p].lut(), want.lut(), err_msg="%s plane %d" % (msg, p))
                np.testing.assert_array_equal(flags[p], c["flags"][p], err_msg="%s plane %d" % (msg, p))
            if c["out"] is not None:
                inp = c["rec"][p][:c["out"][p].shape[0], :c["out"][p].shape[1]].astype(np.uint8)
                got = oracle.ccso_apply_plane(ext, 8, p, inp, prms[p], flags[p])
                np.testing.assert_array_equal(got, c["out"][p], err_msg="%s plane %d" % (msg, p))
