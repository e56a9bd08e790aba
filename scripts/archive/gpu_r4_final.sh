#!/bin/bash
# Round-4 final run: tiled tests, the whole -m gpu suite, smoke, the default bench (the driver's command), then the PMC
# passes behind profiles/r04/pmc/kernels.json, into gpurun_out/$1.  Each GPU step under its own time limit; stop at the
# first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r4final}
mkdir -p $O
export TMPDIR=/tmp
SKIP_TILED= QUICK= NO_BENCH=1 bash scripts/gpu_r4_check.sh ${1:-r4final} || exit 1
timeout -k 10 420 python bench.py > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["frac"], {k: v.get("projected_Mpx_s") for k, v in d["config"]["tile_projection"].items() if k != "note"})'
PROF_OUT=${1:-r4final}/prof bash scripts/pmc_r04.sh || exit 1
echo done
