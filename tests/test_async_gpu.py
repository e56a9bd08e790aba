"""The asynchronous frame-level path (no host round trip inside a frame).

* svtgpu_dlf_pick_async: the FULL_IMAGE bisection of search_filter_level (EbDeblockingFilter.c:886-991) on the device --
  dlf_search_init_kernel, trial rounds whose last workgroup takes the step (dlf_trial_dev_kernel), dlf_finish_kernel --
  and the frame filter with the device levels (svtgpu_dlf_frame_to with NULL parameters), the levels read back at the
  end (svtgpu_dlf_read_levels);
* svtgpu_lr_search_frame_async: the search, the records and rest_finish_search on the device (lr_fin_*_kernel) and the
  apply with the device units (svtgpu_lr_apply_frame with NULL frame types), frame types and units read back at the end.
Run on the reference's pipeline goldens (tests/pipeline_run.py with SVTGPU_TEST_ASYNC=1, in a child process: the
switches are read once per process): the levels, the CDEF stage it feeds, the LR frame types / units and every output
plane bit-exact against the reference.  SVTGPU_DLF_ROUNDS=1 / 3 enqueue fewer trial rounds than the searches take, so
dlf_finish_kernel completes them (one workgroup looping the rounds' items): still bit-exact."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import sys
sys.path[:0] = [%r, %r, %r, %r]
import torch
if torch.cuda.is_available():
    torch.cuda.init()
import pipeline_run as prun
for case in %r:
    prun.check(case, prun.run_gpu(case), "async path")
print("ok")
"""


def _child(cases, **env):
    code = CHILD % (ROOT, os.path.join(ROOT, "svt-av1_pro-anchor-v2.1.0-_amd"), os.path.join(ROOT, "oracle"),
                    os.path.join(ROOT, "tests"), tuple(cases))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=400,
                       env=dict(os.environ, SVTGPU_TEST_ASYNC="1", **env))
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stderr[-3000:]


@pytest.mark.gpu
@pytest.mark.timeout(450)
def test_async_pipeline_bit_exact():
    _child(("mini8", "mini10", "mini10b", "mini8c", "mini8d", "mini10e", "sb128_10", "sbdlf10", "reffs_10",
            "c1_1080p8", "c3_4k10"))


@pytest.mark.gpu
@pytest.mark.timeout(450)
@pytest.mark.parametrize("rounds,cases", [("1", ("mini8", "mini10", "mini10b")), ("3", ("mini8c", "mini10e"))])
def test_async_dlf_finisher_completes_search(rounds, cases):
    _child(cases, SVTGPU_DLF_ROUNDS=rounds)
