"""LPF_PICK_FROM_Q levels (svt_av1_pick_filter_level_by_q, EbDeblockingFilter.c:1036, and qp_based_dlf_param, :992)
against the reference itself: tests/golden/dlf_byq.bin holds 640 cases run through the reference's own
svt_av1_pick_filter_level(LPF_PICK_FROM_Q) by oracle/ref_harness/gen_golden_pipe.c (bit depths 8/10/12, every
qindex class, key/inter frames, I/P/B slices, both temporal-layer indices, every resolution class and zero-strength
level, 1..64 SB ME distortions incl. u32 wrap-around, 0..4 listed references with compound pairs mixed in).
Host logic of libsvtgpu (no device work), so it runs in the CPU suite."""
import numpy as np

import cdef_cases as cc
import svtgpu


def _refs(v):
    """The single-reference levels the reference reads for case row v (duplicates see the last levels written)."""
    levels = {}
    for k in range(int(v[9])):
        t, pk = int(v[10 + k]), int(v[14 + k]) & 0xFFFFFFFF
        if t < 8:
            levels[t] = [(pk >> (8 * j)) & 255 for j in range(4)]
    return [levels[int(v[10 + k])] for k in range(int(v[9])) if int(v[10 + k]) < 8]


def test_ac_quant_table_matches_reference():
    g = cc.load("dlf_byq.bin")
    # the library's table is exercised through qp_based_dlf_param: every qindex of every bit depth
    for b, bd in enumerate((8, 10, 12)):
        for q in range(256):
            y, uv = svtgpu.dlf_qp_based_param(bd, q, 1)
            aq = int(g["ac_quant"][b][q])
            if bd == 8:
                guess = (aq * 6017 + 650707 + (1 << 17)) >> 18
            elif bd == 10:
                guess = (aq * 20723 + 4060632 + (1 << 19)) >> 20
            else:
                guess = (aq * 20723 + 16242526 + (1 << 21)) >> 22
            guess = guess - 2 if guess > 2 else guess - 1 if guess > 1 else guess
            assert y == min(max(guess, 0), 63), (bd, q)


def test_pick_filter_level_by_q_vs_reference():
    g = cc.load("dlf_byq.bin")
    vin, sad, vout = g["in"], g["me_sad"], g["out"]
    bad = []
    for n in range(len(vin)):
        v = [int(x) for x in vin[n]]
        got = svtgpu.dlf_pick_by_q(v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7], sad[n][:v[8]], _refs(v))
        qp = svtgpu.dlf_qp_based_param(v[0], v[1], v[2])
        if list(got) + list(qp) != [int(x) for x in vout[n]]:
            bad.append((n, got, qp, list(vout[n])))
    assert not bad, bad[:5]
    # the sweep reaches every branch: zeroed levels, non-zero levels, the reference-off rule
    assert (vout[:, 0] == 0).sum() > 20 and (vout[:, 0] > 0).sum() > 200 and (vout[:, 2] == 0).sum() > 20
