"""Timeline of the last bench.py step from a rocprofv3 kernel trace: every kernel's start offset, duration and the
idle gap before it, plus idle time per stage.  usage: step_timeline.py <rocprof dir> [last kernel of a step]"""
import csv
import re
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof"
last = sys.argv[2] if len(sys.argv) > 2 else "md_dist"  # the step's final kernel
tr = sorted(csv.DictReader(open(d + "/run_kernel_trace.csv")), key=lambda r: int(r["Start_Timestamp"]))
ends = [i for i, r in enumerate(tr) if last in r["Kernel_Name"]]
seq = tr[ends[-2] + 1:ends[-1] + 1]
t0 = int(seq[0]["Start_Timestamp"])
prev_end = t0
busy = idle = 0
for r in seq:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    m = re.search(r"(\w+)(<[^()]*>)?\(", r["Kernel_Name"])
    name = m.group(1) if m else r["Kernel_Name"][:40]
    gap = max(0, s - prev_end)
    idle += gap
    busy += e - s
    print("%9.1f %8.1f gap %7.1f  %s" % ((s - t0) / 1e3, (e - s) / 1e3, gap / 1e3, name))
    prev_end = max(prev_end, e)
print("step span %.1f us, busy %.1f us, idle %.1f us, %d kernels" % ((prev_end - t0) / 1e3, busy / 1e3, idle / 1e3, len(seq)))
