#!/bin/bash
# Stem variants A/B (tools/stem_probe.py, interleaved): HEAD vs v1 (4-row passes, BN after
# pool) vs v2 (2-row passes, BN after pool); stem tests on v1 and v2.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r02u; mkdir -p $O
L=$R/term-quantization_amd/lib
for rep in 1 2; do for v in old v1 v2; do
  echo -n "$v: "; TQ_LIB_PATH=$L/libtq_hip_$v.so timeout -k 10 120 python tools/stem_probe.py --iters 30 2>&1 | tail -1 || exit 1
done; done
for v in v1 v2; do
  TQ_LIB_PATH=$L/libtq_hip_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_stem.py tests/test_gpu_fused_parity.py -x -q --timeout 200 --timeout-method thread > $O/t_$v.log 2>&1; rc=$?
  echo "$v tests: $(tail -1 $O/t_$v.log)"; [ $rc -ne 0 ] && { tail -30 $O/t_$v.log; exit 1; }
done
exit 0
