#!/bin/bash
# one SQ pass over a short F = 1 bench: LDS instructions and bank-conflict cycles per kernel (gpurun_out/$1)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-lds}
mkdir -p $O
export TMPDIR=/tmp
K="wiener_res|sgr_res|sgr_flt|wiener_stats|wiener_solve|cdef_search|cdef_apply|sod_step|dlf_tile|lr_apply|md_dist"
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_WAVES --kernel-include-regex "$K" -d $O/sq -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-matrix --frames-in-flight 1 --no-kernel-timing > $O/sq.log 2>&1 || { echo "pmc failed"; tail -5 $O/sq.log; exit 1; }
python3 - "$O" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/sq/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(f)):
    n = r["Kernel_Name"].split("(")[0].split("::")[-1][:40]
    acc[n][r["Counter_Name"]] += float(r["Counter_Value"])
for n, v in sorted(acc.items()):
    li = v["SQ_INSTS_LDS"]
    print("%-40s lds %12.0f conflicts/lds %.3f valu %12.0f" % (n, li, v["SQ_LDS_BANK_CONFLICT"] / li if li else 0, v["SQ_INSTS_VALU"]))
PY
