"""Per-frame device time per kernel from a rocprofv3 --kernel-trace --stats summary (run_kernel_stats.csv).
usage: kstats.py <kernel_stats.csv> [frames]   (frames: default = the sgr_flt_kernel launch count, one per frame)"""
import csv
import re
import sys


def main(path, frames=None):
    rows = list(csv.DictReader(open(path)))
    name = lambda r: re.sub(r"^(void )?(\(anonymous namespace\)::)?", "", r["Name"]).split("(")[0]
    if frames is None:
        frames = next((int(r["Calls"]) for r in rows if "sgr_flt_kernel" in r["Name"]), 1)
    tot = 0.0
    print("%-44s %8s %10s %10s" % ("kernel", "calls/fr", "us/frame", "avg us"))
    for r in sorted(rows, key=lambda r: -int(r["TotalDurationNs"])):
        us = int(r["TotalDurationNs"]) / frames / 1e3
        tot += us
        print("%-44s %8.1f %10.1f %10.1f" % (name(r)[:44], int(r["Calls"]) / frames, us, float(r["AverageNs"]) / 1e3))
    print("%-44s %8s %10.1f   (%d frames)" % ("total", "", tot, frames))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else None)
