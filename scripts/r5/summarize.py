"""Summarise a directory of bench logs (one JSON bench line each) into a table: value, LR stage, top kernels.
   python scripts/r5/summarize.py gpurun_out/r5ab2 > profiles/r05/.../summary.txt"""
import glob
import json
import os
import sys

d = sys.argv[1]
for f in sorted(glob.glob(os.path.join(d, "*.log"))):
    lines = [l for l in open(f) if l.startswith("{")]
    stats = [l.strip() for l in open(f) if l.startswith(("sgr_res:", "wiener_res:"))]
    if lines:
        b = json.loads(lines[-1])
        r = b.get("roofline", {})
        k = r.get("all_kernels_ms_per_frame", {})
        top = ", ".join(f"{n} {v:.3f}" for n, v in list(k.items())[:4])
        print(f"{os.path.basename(f):28s} {b['value']:8.1f} {b['unit']}  F={b['config'].get('frames_in_flight')}  "
              f"lr_search_apply {b['config']['stage_ms'].get('lr_search_apply', 0):.3f} ms  [{top}]")
    for s in stats[-2:]:
        print(f"{os.path.basename(f):28s} {s}")
