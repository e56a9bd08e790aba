#!/bin/bash
# Round-6 regression A/B on one box: the round-5 build (a git worktree of ae1aa7f under _ab/r5, its own libsvtgpu.so
# built there) against this tree, alternating, at $CFGS (4K 10-bit and 1080p 10-bit by default), plus this tree with
# the synchronous searches and the host LR finish.  Output: gpurun_out/$1/<cfg>_<variant>_<i>.log + one summary line
# per run.  Each run under its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r6ab}
mkdir -p $O
export TMPDIR=/tmp
STEPS=${STEPS:-40}
COMMON="--no-cpu-baseline --no-matrix --no-tile-projection --host-timing --steps $STEPS --warmup 5"
summ() { grep '^{' $1 | python -c '
import json,sys
d=json.loads(sys.stdin.read()); c=d["config"]
print(d["value"], d["ms_per_step"], "lat", c.get("frame_latency_ms"),
      {k: round(v, 3) for k, v in c["stage_ms"].items() if k != "note"})'; }
declare -A CFG=([4k10]="" [1080p10]="--width 1920 --height 1080 --bit-depth 10")
for R in ${REPS:-1 2}; do
  for C in ${CFGS:-4k10 1080p10}; do
    for V in ${VARIANTS:-r5 cur cursync curhostfin}; do
      # a variant: r5 | cur | curtorch | cursync | curhostfin, optionally ":VAR=v,VAR2=v" (environment of that run)
      B0=${V%%:*}; E=""; [ "$B0" != "$V" ] && E=$(echo "${V#*:}" | tr ',' ' ')
      case $B0 in
        r5) D=_ab/r5; X="" ;;
        cur) D=.; X="" ;;
        curtorch) D=.; X="--torch-streams" ;;
        cursync) D=.; X="--dlf-sync --lr-sync" ;;
        curhostfin) D=.; E="$E SVTGPU_LR_FINISH=host"; X="--dlf-sync --lr-sync" ;;
      esac
      L=$O/${C}_$(echo $V | tr ":=," "___")_${R}.log
      ( cd $D && env $E timeout -k 10 300 python bench.py $COMMON ${CFG[$C]} $X $BENCH_ARGS ) > $L 2>&1 ||
        { echo "bench $C $V failed"; tail -20 $L; exit 1; }
      echo "$C $V #$R: $(summ $L)"
    done
  done
done
echo done
