"""The global-memory mode of the resident Wiener kernel (wiener_res_kernel): units whose CDEF window does not fit the
CU's LDS (no row-part cut up to WR_MAX_PARTS fits) read it and the source from global memory per candidate.  No
frame of the default configurations takes that path, so it runs here on the pipeline goldens with the LDS cap set
to 0 (SVTGPU_WR_LDS_CAP, read once per process: a child process) -- bit-exact against the reference like the
default path (every selectable path under a test)."""
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
for case in ("mini10", "sb128_10", "c3_4k10"):
    prun.check(case, prun.run_gpu(case), "wr global mode")
print("ok")
"""


@pytest.mark.gpu
def test_wiener_global_memory_mode_bit_exact():
    code = CHILD % (ROOT, os.path.join(ROOT, "svt-av1_pro-anchor-v2.1.0-_amd"), os.path.join(ROOT, "oracle"),
                    os.path.join(ROOT, "tests"))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, SVTGPU_WR_LDS_CAP="0"))
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stderr[-3000:]


CHILD_SR = r"""
import sys
sys.path[:0] = [%r, %r, %r, %r]
import torch
if torch.cuda.is_available():
    torch.cuda.init()
import pipeline_run as prun
for case in ("mini10", "mini8", "sb128_10", "mini10e"):
    prun.check(case, prun.run_gpu(case), "sr parts")
print("ok")
"""


@pytest.mark.gpu
def test_sgr_resident_row_parts_bit_exact():
    """The resident self-guided search (sgr_res_kernel) cuts units larger than one CU's registers into row parts whose
    moments and candidate errors meet through uncached memory every pass; at the default part size only the 4K
    frame's bottom luma unit row takes that path (2 parts, c3_4k10 in the pipeline goldens).  With the part size
    lowered to 4096 pixels (SVTGPU_SR_PART_PX, read once per process: a child process) the small cases' units run as
    2-6 parts each -- bit-exact against the reference like the whole-unit path."""
    code = CHILD_SR % (ROOT, os.path.join(ROOT, "svt-av1_pro-anchor-v2.1.0-_amd"), os.path.join(ROOT, "oracle"),
                       os.path.join(ROOT, "tests"))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, SVTGPU_SR_PART_PX="4096"))
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stderr[-3000:]


CHILD_TREE = r"""
import sys
sys.path[:0] = [%r, %r, %r, %r]
import torch
if torch.cuda.is_available():
    torch.cuda.init()
import pipeline_run as prun
for case in ("mini10", "mini8d", "sb128_10", "sbdlf10"):
    prun.check(case, prun.run_gpu(case), "sr tree")
print("ok")
"""


@pytest.mark.gpu
@pytest.mark.parametrize("nodes", ["3", "7"])
def test_sgr_resident_speculative_trees_bit_exact(nodes):
    """The resident self-guided search evaluates one candidate per pass by default; SVTGPU_SR_TREE=3 / 7 evaluate a
    complete speculative outcome tree per pass (each node built by one control lane from the root's state along its
    path) -- fewer passes, the same decisions: bit-exact against the reference."""
    code = CHILD_TREE % (ROOT, os.path.join(ROOT, "svt-av1_pro-anchor-v2.1.0-_amd"), os.path.join(ROOT, "oracle"),
                         os.path.join(ROOT, "tests"))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, SVTGPU_SR_TREE=nodes))
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stderr[-3000:]
