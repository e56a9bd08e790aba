"""Per-launch HBM-side traffic of each kernel from scripts/pmc_traffic.sh's two rocprofv3 passes -> JSON for bench.py.

traffic = 2 x FETCH_SIZE + WRITE_SIZE (bytes; the counters are in KB).  The factor 2 is the gfx950 correction of
MI355X_MICROARCH.md (HBM section): FETCH_SIZE tallies 128-B read requests at 64 B.  fetch_cal (scripts/ubench) checks
it on this box for 2-, 4-, 8- and 16-byte lanes (FETCH_SIZE = exactly 1/2 of a known 1 GiB read) and WRITE_SIZE = the
bytes of a 16-B-lane store; both calibration ratios are recorded in the output.
usage: pmc_traffic.py <gpurun_out/traffic> <out.json>
"""
import collections
import csv
import json
import os
import re
import sys


def per_kernel(path):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    ids = collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        m = re.search(r"(\w+)(<[^()]*>)?\(", r["Kernel_Name"])
        k = (m.group(1) + (m.group(2) or "")) if m else r["Kernel_Name"][:40]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        ids[k].add(r["Dispatch_Id"])
    return {k: {c: x / len(ids[k]) for c, x in v.items()} | {"launches": len(ids[k])} for k, v in agg.items()}


def main(d, out):
    f = per_kernel(os.path.join(d, "bench_fetch", "run_counter_collection.csv"))
    w = per_kernel(os.path.join(d, "bench_write", "run_counter_collection.csv"))
    cf = per_kernel(os.path.join(d, "cal_fetch", "run_counter_collection.csv"))
    cw = per_kernel(os.path.join(d, "cal_write", "run_counter_collection.csv"))
    gib_kb = float(1 << 20)
    cal = {"read_%dB_lane" % n: cf.get("read_w<%s>" % t, {}).get("FETCH_SIZE", 0) / gib_kb
           for n, t in ((2, "unsigned short"), (4, "unsigned int"), (8, "HIP_vector_type<unsigned int, 2u> "),
                        (16, "HIP_vector_type<unsigned int, 4u> "))}
    cal.update({
           "write_16B_lane": cw.get("write_16", {}).get("WRITE_SIZE", 0) / gib_kb})
    res = {"method": "2 x FETCH_SIZE + WRITE_SIZE per launch (bytes), separate rocprofv3 --pmc passes over "
                     "bench.py --steps 2 --warmup 1; FETCH_SIZE x 2 per the gfx950 correction",
           "calibration_counter_per_byte": cal, "kernels": {}}
    for k in sorted(set(f) & set(w)):
        fb, wb = f[k]["FETCH_SIZE"] * 1024, w[k]["WRITE_SIZE"] * 1024
        res["kernels"][k] = {"launches": f[k]["launches"], "fetch_size_bytes": round(fb), "write_size_bytes": round(wb),
                             "traffic_bytes": round(2 * fb + wb)}
    json.dump(res, open(out, "w"), indent=1)
    for k, v in res["kernels"].items():
        print("%-28s %5d  traffic %.3g B/launch" % (k, v["launches"], v["traffic_bytes"]))
    print(cal)


if __name__ == "__main__":
    main(*sys.argv[1:3])
