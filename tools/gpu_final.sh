#!/bin/bash
# dw checks (tools/gpu_dw.sh) then the round check (tools/gpu_round.sh); the second runs
# only if the first ended normally (exit 0, or 1 = a failed assertion, not a fault/timeout)
set -u
bash tools/gpu_dw.sh ${1:-dw}
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "dw step rc=$rc: stopping"; exit $rc; fi
bash tools/gpu_round.sh ${2:-round}
