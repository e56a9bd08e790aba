"""Diagnostic: the LR device finish's phase times (SVTGPU_LR_FIN_CLK) on the pinned 4K 10-bit and 1080p 8-bit cases
(synchronous search: the clocks are printed at the collect).  python scripts/r6/finclk.py"""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "svt-av1_pro-anchor-v2.1.0-_amd"), os.path.join(ROOT, "oracle"),
                os.path.join(ROOT, "tests")]
os.environ["SVTGPU_LR_FIN_CLK"] = "1"
import pipeline_run as prun  # noqa: E402
for case in sys.argv[1:] or ("c3_4k10", "c1_1080p8"):
    for _ in range(3):
        prun.check(case, prun.run_gpu(case, async_=False), "finclk")
    print(case, "ok", flush=True)
