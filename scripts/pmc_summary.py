"""Per-kernel averages of a rocprofv3 --pmc counter collection (one line per kernel)."""
import collections
import csv
import re
import sys

for f in sys.argv[1:]:
    rows = list(csv.DictReader(open(f)))
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    ids = collections.defaultdict(set)
    for r in rows:
        m = re.search(r"::(\w+)(<[^>]*>)?\(", r["Kernel_Name"])
        k = (m.group(1) + (m.group(2) or "")) if m else r["Kernel_Name"][:40]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        ids[k].add(r["Dispatch_Id"])
    for k, v in agg.items():
        n = len(ids[k])
        print(k, n, {c: "%.3g" % (x / n) for c, x in sorted(v.items())})
