#!/bin/bash
# (STEM_HELP was a timing-only build option, reverted after this probe: profiles/r05_stem_trace.txt)
# Stem SIMD-partner epilogue help A/B (STEM_HELP variant builds help / helptr): parity of the
# help build (tests/test_gpu_stem.py), then per-tile phases + per-wave lag (tools/stem_trace.py)
# and kernel time (tools/stem_probe.py) against the product build, two rounds.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"
TQ_LIB_PATH=$R/term-quantization_amd/lib/libtq_hip_help.so timeout -k 10 300 \
  python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_stem.py \
  > gpurun_out/help_parity.log 2>&1 || { tail -30 gpurun_out/help_parity.log; exit 1; }
tail -3 gpurun_out/help_parity.log
for r in 1 2; do
  for v in basetr helptr; do
    export TQ_LIB_PATH=$R/term-quantization_amd/lib/libtq_hip_$v.so
    echo "== round $r $v"
    timeout -k 10 120 python tools/stem_trace.py 2>&1 | grep -v amdgpu.ids || exit 1
  done
  for v in libtq_hip libtq_hip_help; do
    export TQ_LIB_PATH=$R/term-quantization_amd/lib/$v.so
    echo "== round $r $v"
    timeout -k 10 120 python tools/stem_probe.py --iters 30 2>&1 | grep stem || exit 1
  done
done
