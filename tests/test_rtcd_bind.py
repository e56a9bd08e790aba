"""The drop-in boundary, end to end: the reference's own frame code with its RTCD function pointers bound to the
libsvtgpu shims.

oracle/_ref/rtcd_pipe is oracle/ref_harness/gen_golden_pipe.c compiled against the reference headers with
-DSVTGPU_BIND and -Werror=incompatible-pointer-types: every shim (loop filter x16, CDEF filter / 8xn / find_dir /
dist / search_one_dual / copy_rect8, Wiener and self-guided filters, compute_stats, pixel_proj_error,
get_proj_subspace, mse16x16, the full-distortion kernels; and, compile-only, the ME / MD distortion / frame-buffer
shims: sad / x4d / variance / highbd variance / sub-pixel variance of all sizes, sse, nxm SAD, the open-loop ME and
MD full-pel search kernels, the 8 <-> 16-bit conversions, padding, frame extension) is assigned to the reference's
pointer without a cast,
and svt_av1_pick_filter_level, svt_av1_loop_filter_frame, cdef_seg_search / finish_cdef_search /
svt_av1_cdef_frame, restoration_seg_search / rest_finish_search / svt_av1_loop_restoration_filter_frame then run
through the device.  Every output must equal the pure-C run of the same code (tests/golden/pipe_<case>.npz)."""
import os
import subprocess
import tempfile

import numpy as np
import pytest

import golden_io
import pipeline_cases as pc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RTCD_PIPE = os.path.join(ROOT, "oracle", "_ref", "rtcd_pipe")
CASES = ["mini10b", "mini8c"]  # few CDEF strengths: the per-block shims are synchronous round trips


@pytest.mark.gpu
@pytest.mark.skipif(not os.path.exists(RTCD_PIPE), reason="oracle/_ref/rtcd_pipe not built (needs /root/reference)")
@pytest.mark.parametrize("case", CASES)
def test_reference_frame_code_through_device_shims(case):
    src, rec, mi = pc.inputs(case)
    g = pc.load(case)
    with tempfile.TemporaryDirectory() as td:
        fin, fout = os.path.join(td, "in.bin"), os.path.join(td, "out.bin")
        pc.write_input(fin, case, src, rec, mi)
        res = subprocess.run([RTCD_PIPE, "pipe", fin, fout], capture_output=True, text=True, timeout=280)
        assert res.returncode == 0, res.stderr[-2000:]
        out = golden_io.load(fout)
    # the statistics record (wn_stats_*) comes from the pure-C run's recording kernels only
    keys = set(k for k in g if k != "input_sha" and not k.startswith("wn_stats_"))
    assert keys <= set(out), sorted(keys - set(out))
    for k in sorted(keys):
        a, b = np.array(out[k]), np.array(g[k])
        if k.startswith("lr_units"):  # {type, vfilter[8], hfilter[8], ep, xqd[2]}: the fields of the unused filter
            for arr in (a, b):     # are whatever RestorationUnitInfo held before (uninitialised in the reference)
                arr[arr[:, 0] != 1, 1:17] = 0
                arr[arr[:, 0] != 2, 17:20] = 0
        np.testing.assert_array_equal(a, b, err_msg="%s: %s differs between the C and the device-shim runs" % (case, k))


@pytest.mark.skipif(not os.path.isdir("/root/reference/Source"), reason="reference headers not present")
def test_shim_prototypes_match_reference_pointers():
    """CPU, compile-only: include/svtgpu.h against the reference's RTCD headers under -Werror=incompatible-pointer-types
    and -Werror=discarded-qualifiers (oracle/ref.mk bindcheck)."""
    r = subprocess.run(["make", "-s", "-f", "oracle/ref.mk", "bindcheck"], cwd=ROOT, capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]


RTCD_INSTALL = os.path.join(ROOT, "oracle", "_ref", "rtcd_install")


@pytest.mark.skipif(not os.path.exists(RTCD_INSTALL), reason="oracle/_ref/rtcd_install not built (needs /root/reference)")
def test_install_point_before_init_fn_ptr():
    """The install point of include/svtgpu_rtcd.h: the reference's init_fn_ptr (av1me.c:31, called
    at EbEncHandle.c:1546) copies the 110 sad / x4d / variance / highbd variance / sub-pixel variance pointers of the 22
    block sizes into svt_aom_mefn_ptr[], which ME and MD call.  Installed between the RTCD setup (:1531) and that
    call, every entry is a libsvtgpu shim; installed after it, none is.  Pointer comparisons only (CPU)."""
    res = subprocess.run([RTCD_INSTALL], capture_output=True, text=True, timeout=60)
    assert res.returncode == 0, res.stderr[-2000:]
    assert res.stdout.split() == ["documented", "110/110", "late", "0/110"], res.stdout
