#!/bin/bash
# stream-split parity tests, then the profile session at the new bench defaults (2 streams, graph)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r02s; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused_parity.py -x -v --timeout 300 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -6 $O/t.log
bash tools/gpu_profile.sh r02s
