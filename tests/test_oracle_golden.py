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
    for lvl in (0, 11, 14, 15, 17):
        with pytest.raises(ValueError):
            oracle.controls(lvl)


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
        got = oracle.dlf_frame(c["inp"], c["bd"], c["mi"], c["params"], c["plane_start"], c["plane_end"])
        for p in range(3):
            assert np.array_equal(got[p], c["out"][p]), (c["name"], p)
        n += 1
    assert n >= 8
