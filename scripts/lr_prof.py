"""Summarise a rocprofv3 kernel trace of bench.py: top kernels and the per-round LR search launch durations."""
import csv
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof"
rows = list(csv.DictReader(open(d + "/run_kernel_stats.csv")))
for r in rows[:14]:
    print(r["Name"][:70].ljust(70), r["Calls"], r["AverageNs"][:10], r["Percentage"][:6])
tr = list(csv.DictReader(open(d + "/run_kernel_trace.csv")))


def dur(name, n):
    return [round((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000) for r in tr if name in r["Kernel_Name"]][-n:]


for k, n in (("wiener_trial", 40), ("proj_err", 16), ("wiener_advance", 41), ("sgr_advance", 17)):
    print(k, dur(k, n))
