#!/bin/bash
# (AEA_UNROLL / AEA_F32Q were timing-only build options, reverted after this probe: profiles/r05_aea_ab.txt)
# act_encode_act fp32-quotient A/B (AEA_F32Q variant build f32q): parity of each build
# (the effnet fused tests + test_gpu_fused's act_encode_act cases), then tools/aea_probe.py.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"
for v in libtq_hip libtq_hip_f32q; do
  TQ_LIB_PATH=$R/term-quantization_amd/lib/$v.so timeout -k 10 300 \
    python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_fused_effnet.py tests/test_gpu_fused.py -k "effnet or act_encode or lut or swish" \
    > gpurun_out/aea_parity_$v.log 2>&1 || { tail -30 gpurun_out/aea_parity_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/aea_parity_$v.log)"
done
for r in 1 2; do for v in libtq_hip libtq_hip_f32q; do
  echo "== round $r $v"
  TQ_LIB_PATH=$R/term-quantization_amd/lib/$v.so timeout -k 10 120 python tools/aea_probe.py \
    2>&1 | grep aea || exit 1
done; done
