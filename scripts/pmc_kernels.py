"""Per-launch PMC figures of each kernel from scripts/pmc_r03.sh's rocprofv3 passes -> the JSON bench.py reads.

traffic = 2 x FETCH_SIZE + WRITE_SIZE (bytes; the counters are in KB).  The factor 2 is the gfx950 correction of
MI355X_MICROARCH.md (HBM section): FETCH_SIZE tallies 128-B read requests at 64 B; fetch_cal checks it on the box for
2-, 4-, 8- and 16-byte lanes (FETCH_SIZE = exactly 1/2 of a known 1 GiB read) and WRITE_SIZE = the bytes of a 16-B-lane
store; both calibration ratios are recorded.  SQ counters are per launch (summed over the chip).
usage: pmc_kernels.py <gpurun_out/r03prof> <out.json>
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
    cc = lambda sub: os.path.join(d, sub, "run_counter_collection.csv")
    f, w = per_kernel(cc("bench_fetch")), per_kernel(cc("bench_write"))
    sq = {}
    for part in ("sqA", "sqB"):
        for k, v in per_kernel(cc(part)).items():
            sq.setdefault(k, {}).update({c: x for c, x in v.items() if c != "launches"})
    cf, cw = per_kernel(cc("cal_fetch")), per_kernel(cc("cal_write"))
    gib_kb = float(1 << 20)
    cal = {"read_%dB_lane" % n: cf.get("read_w<%s>" % t, {}).get("FETCH_SIZE", 0) / gib_kb
           for n, t in ((2, "unsigned short"), (4, "unsigned int"), (8, "HIP_vector_type<unsigned int, 2u> "),
                        (16, "HIP_vector_type<unsigned int, 4u> "))}
    cal["write_16B_lane"] = cw.get("write_16", {}).get("WRITE_SIZE", 0) / gib_kb
    res = {"method": "2 x FETCH_SIZE + WRITE_SIZE per launch (bytes) and SQ counters per launch, separate rocprofv3 "
                     "--pmc passes over bench.py --steps 2 --warmup 1 --frames-in-flight 1 --no-tile-projection (full 4K frames "
                     "only); FETCH_SIZE x 2 per the "
                     "gfx950 correction",
           "calibration_counter_per_byte": cal, "kernels": {}}
    for k in sorted(set(f) & set(w)):
        fb, wb = f[k]["FETCH_SIZE"] * 1024, w[k]["WRITE_SIZE"] * 1024
        e = {"launches": f[k]["launches"], "fetch_size_bytes": round(fb), "write_size_bytes": round(wb),
             "traffic_bytes": round(2 * fb + wb)}
        e.update({c: round(x, 1) for c, x in sorted(sq.get(k, {}).items())})
        if e.get("SQ_INSTS_LDS"):
            e["lds_conflict_cycles_per_lds_inst"] = round(e.get("SQ_LDS_BANK_CONFLICT", 0) / e["SQ_INSTS_LDS"], 3)
        if e.get("SQ_WAVE_CYCLES"):
            e["wait_any_frac"] = round(e.get("SQ_WAIT_ANY", 0) / e["SQ_WAVE_CYCLES"], 3)
        res["kernels"][k] = e
    json.dump(res, open(out, "w"), indent=1)
    for k, v in res["kernels"].items():
        print("%-40s %4d  traffic %.3g B  valu %.3g  lds-conf/inst %s" % (k, v["launches"], v["traffic_bytes"],
              v.get("SQ_INSTS_VALU", 0), v.get("lds_conflict_cycles_per_lds_inst")))
    print(cal)


if __name__ == "__main__":
    main(*sys.argv[1:3])
