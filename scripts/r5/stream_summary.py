"""Bytes per launch (2 x FETCH_SIZE + WRITE_SIZE, KB units per the gfx950 correction) and average duration of the
streaming kernels from scripts/r5/stream_ab.sh's output.  usage: stream_summary.py <dir> <tag>"""
import csv
import os
import re
import sys
from collections import defaultdict


def short(n):
    m = re.search(r"(\w+_kernel)(<[^>]*>)?", n)
    return (m.group(1) + (m.group(2) or "")) if m else n[:40]


def counters(path):
    acc = defaultdict(list)
    for r in csv.DictReader(open(path)):
        acc[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main(d, t):
    f = counters(os.path.join(d, t + "_fetch", "run_counter_collection.csv"))
    w = counters(os.path.join(d, t + "_write", "run_counter_collection.csv"))
    dur = {}
    for r in csv.DictReader(open(os.path.join(d, t + "_trace", "run_kernel_stats.csv"))):
        dur[short(r["Name"])] = float(r["AverageNs"]) / 1e3
    for k in sorted(f):
        mb = (2 * f[k] + w.get(k, 0)) * 1024 / 1e6
        us = dur.get(k)
        print("%s %-34s traffic %7.1f MB  (fetch %6.1f write %6.1f)  avg %s us" %
              (t, k, mb, 2 * f[k] * 1024 / 1e6, w.get(k, 0) * 1024 / 1e6, "%.1f" % us if us else "-"))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
