#!/bin/bash
# Stem: 16 waves (two per strip, channel halves) vs the committed 8-wave kernel (v1).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r02z; mkdir -p $O
L=$R/term-quantization_amd/lib
timeout -k 10 300 python -u -m pytest tests/test_gpu_stem.py -x -q --timeout 200 --timeout-method thread > $O/t.log 2>&1; rc=$?
tail -2 $O/t.log; [ $rc -ne 0 ] && { grep -E "Error|assert" $O/t.log | head; exit $rc; }
for rep in 1 2; do for v in new v1 tp2; do
  if [ $v = v1 ]; then export TQ_LIB_PATH=$L/libtq_hip_ab.so; else unset TQ_LIB_PATH; fi
  if [ $v = tp2 ]; then export TQ_STEM_TP=2; else unset TQ_STEM_TP; fi
  echo -n "$v: "; timeout -k 10 120 python tools/stem_probe.py --iters 30 2>&1 | tail -1 || exit 1
done; done
