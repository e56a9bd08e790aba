#!/bin/bash
# Kernel-trace statistics of the round-5 build (_ab/r5, see ab_r5.sh) against this tree on one box: the same bench
# flags ($ARGS; default 1080p 10-bit, 4 frames in flight, both searches synchronous in this tree), into
# gpurun_out/$1/{r5,cur}/.  Each run under its own time limit; prints the kernels' totals side by side.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=$PWD/gpurun_out/${1:-r6profab}
mkdir -p $O/r5 $O/cur
export TMPDIR=/tmp
ARGS=${ARGS:---width 1920 --height 1080 --bit-depth 10 --frames-in-flight 4}
B="--no-cpu-baseline --no-matrix --no-tile-projection --no-kernel-timing --steps ${STEPS:-20} --warmup 3 $ARGS"
for V in r5 cur; do
  D=.; X="--dlf-sync --lr-sync"
  [ $V = r5 ] && D=_ab/r5 && X=""
  ( cd $D && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/$V -o run --output-format csv -- python3 bench.py $B $X ) \
      > $O/$V/bench.log 2>&1 || { echo "profile $V failed"; tail -20 $O/$V/bench.log; exit 1; }
  echo "$V: $(grep '^{' $O/$V/bench.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["frame_latency_ms"])')"
done
python3 - $O/r5 $O/cur <<'PY'
import csv, glob, sys
def load(d):
    f = glob.glob(d + "/**/*kernel_stats.csv", recursive=True)[0]
    return {r["Name"]: (int(r["Calls"]), float(r["TotalDurationNs"]) / 1e6) for r in csv.DictReader(open(f))}
a, b = load(sys.argv[1]), load(sys.argv[2])
names = sorted(set(a) | set(b), key=lambda k: -max(a.get(k, (0, 0))[1], b.get(k, (0, 0))[1]))
print("%-64s %14s %14s" % ("kernel", "r5 calls/ms", "cur calls/ms"))
for k in names[:30]:
    x, y = a.get(k, (0, 0.0)), b.get(k, (0, 0.0))
    print("%-64s %5d %8.2f %5d %8.2f" % (k[:64], x[0], x[1], y[0], y[1]))
print("total ms: r5 %.2f cur %.2f" % (sum(v[1] for v in a.values()), sum(v[1] for v in b.values())))
PY
echo done
