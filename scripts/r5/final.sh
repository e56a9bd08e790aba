#!/bin/bash
# Round-end state on one GPU box, in two gpurun calls (each well inside gpurun's limit):
#   bash scripts/r5/final.sh check <out>   the whole -m gpu suite, smoke(), the driver's default bench
#   bash scripts/r5/final.sh prof  <out>   FETCH/WRITE calibration + PMC passes + kernel traces at F = 1 / 4
#                                          (scripts/r5/pmc_r05.sh; summarised by scripts/pmc_kernels.py into kernels.json)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
case "$1" in
  check) SMOKE=1 bash scripts/r5/check.sh "${2:-r5final}" ;;
  prof)  PROF_OUT="${2:-r5prof}" bash scripts/r5/pmc_r05.sh ;;
  *) echo "usage: final.sh check|prof [out]"; exit 2 ;;
esac
