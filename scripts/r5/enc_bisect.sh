#!/bin/bash
# Which frame-level stage makes a frame-hook encode differ from the encoder as built: the clip encoded on the CPU, then
# with the hooks of one stage at a time (ENC_HOOK_STAGES bits 1 DLF, 2 CDEF, 4 LR).  GEOM="w h frames preset qp".
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r5encb}
mkdir -p $O
E=oracle/_ref/enc/enc_drop_in
G=${GEOM:-250 138 3 2 40}
timeout -k 10 300 $E cpu $O/cpu.obu $G > $O/cpu.log 2>&1 || { echo "cpu encode failed"; tail $O/cpu.log; exit 1; }
for m in ${STAGES:-1 2 4 7}; do
  ENC_HOOK_STAGES=$m timeout -k 10 300 $E frame $O/s$m.obu $G > $O/s$m.log 2>&1 || { echo "stage $m encode failed"; tail $O/s$m.log; exit 1; }
  if cmp -s $O/cpu.obu $O/s$m.obu; then r=same; else r=DIFFERS; fi
  echo "stages $m: $r ($(grep -E '^frame (bytes|kinds)' $O/s$m.log | tr '\n' ' '))"
done
