"""Timeline of one bench.py step from a rocprofv3 kernel trace: every kernel's start offset, duration, queue and the
idle gap of the device before it.  A step starts at an occurrence of the `first` kernel (default: the DLF trial).
usage: step_timeline.py <rocprof dir> [first kernel of a step] [which step from the end, default 2]"""
import csv
import re
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof"
first = sys.argv[2] if len(sys.argv) > 2 else "dlf_tile_kernel<unsigned short, true>"
back = int(sys.argv[3]) if len(sys.argv) > 3 else 2
tr = sorted(csv.DictReader(open(d + "/run_kernel_trace.csv")), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(tr) if first in r["Kernel_Name"] and (i == 0 or first not in tr[i - 1]["Kernel_Name"])]
seq = tr[starts[-back]:starts[-back + 1]] if back > 1 else tr[starts[-1]:]
t0 = int(seq[0]["Start_Timestamp"])
prev_end = t0
busy = idle = 0
per = {}
for r in seq:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    m = re.search(r"(\w+)(<[^()]*>)?\(", r["Kernel_Name"])
    name = m.group(1) if m else r["Kernel_Name"][:40]
    gap = max(0, s - prev_end)
    idle += gap
    busy += e - s
    per[name] = per.get(name, 0) + (e - s)
    print("%9.1f %8.1f gap %7.1f q%s %s" % ((s - t0) / 1e3, (e - s) / 1e3, gap / 1e3, r["Queue_Id"], name))
    prev_end = max(prev_end, e)
print("step span %.1f us, device idle %.1f us, %d kernels" % ((prev_end - t0) / 1e3, idle / 1e3, len(seq)))
for k, v in sorted(per.items(), key=lambda kv: -kv[1]):
    print("  %8.1f us  %s" % (v / 1e3, k))
