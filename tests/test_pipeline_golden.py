"""Whole-frame pipeline parity against the reference's own frame-level code (tests/golden/pipe_*.npz, made by
tests/golden/make_pipeline_golden.py with oracle/_ref/gen_golden_pipe).

CPU (not gpu): the oracle restatement runs the small SB64 cases end to end — DLF level pick + filter, CDEF
search / strength pick / apply, LR search / apply — and must reproduce every reference output bit for bit; the
control tables of libsvtgpu must equal the reference's EncModeConfig.c tables.
GPU: libsvtgpu runs every case, including the 1080p 8-bit and 4K 10-bit configurations (digests).
"""
import ctypes

import numpy as np
import pytest

import pipeline_cases as pc
import pipeline_run as pr

@pytest.mark.parametrize("case", pc.SMALL)
def test_pipeline_inputs_stable(case):
    """The integer-only input generator reproduces the inputs the fixture was made from."""
    src, rec, mi = pc.inputs(case)
    assert pc.input_digest(src, rec, mi) == str(pc.load(case)["input_sha"])


@pytest.mark.parametrize("case", pc.SMALL)
def test_oracle_pipeline_vs_reference(case):
    pr.check(case, pr.run_oracle(case), "oracle")


def test_cdef_controls_vs_reference_tables():
    import svtgpu
    for level in range(18):
        ref = pr.ctrl_tables()["cdef"][level]
        c = svtgpu.CdefControls()
        rc = svtgpu.lib().svtgpu_cdef_controls_for_level(level, ctypes.byref(c))
        if not ref[0]:
            assert rc != 0, level  # CDEF off: no search controls
            continue
        assert rc == 0, level
        n1, n2 = int(ref[1]), int(ref[2])
        assert (c.first_pass_fs_num, c.default_second_pass_fs_num, c.subsampling_factor, c.zero_fs_cost_bias) == \
            (n1, n2, ref[5], ref[6]), level
        assert list(c.default_first_pass_fs[:n1]) == list(ref[8:8 + n1]), level
        assert list(c.default_second_pass_fs[:n2]) == list(ref[72:72 + n2]), level
        assert list(c.default_first_pass_fs_uv[:n1]) == list(ref[136:136 + n1]), level
        assert list(c.default_second_pass_fs_uv[:n2]) == list(ref[200:200 + n2]), level
        assert int(c.use_reference_cdef_fs) == int(ref[3]), level


def test_lr_controls_vs_reference_tables():
    import svtgpu
    t = pr.ctrl_tables()
    for wn in range(6):
        for sg in range(5):
            c = svtgpu.LrSearchControls()
            assert svtgpu.lib().svtgpu_lr_controls_for_level(wn, sg, ctypes.byref(c)) == 0
            w, s = t["wn"][wn], t["sg"][sg]
            assert c.wn_enabled == w[0] and c.sg_enabled == s[0], (wn, sg)
            if w[0]:
                assert (c.wn_filter_tap_lvl, c.wn_use_refinement, c.wn_max_one_refinement_step, c.wn_use_chroma) == \
                    tuple(int(x) for x in (w[1], w[2], w[3], w[5])), wn
            if s[0]:
                assert c.sg_use_chroma == s[2], sg
                assert (list(c.sg_start_ep), list(c.sg_end_ep), list(c.sg_ep_inc), list(c.sg_refine)) == \
                    ([int(x) for x in s[3:5]], [int(x) for x in s[5:7]], [int(x) for x in s[7:9]],
                     [int(x) for x in s[9:11]]), sg


@pytest.mark.gpu
@pytest.mark.parametrize("case", list(pc.CASES))
def test_gpu_pipeline_vs_reference(case):
    pr.check(case, pr.run_gpu(case), "gpu")
