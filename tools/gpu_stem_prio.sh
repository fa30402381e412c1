#!/bin/bash
# (STEM_PRIO was a timing-only build option, reverted after this probe: profiles/r05_stem_trace.txt)
# Stem wave-priority A/B (STEM_PRIO variant builds sp1 / sp2, all with STEM_TRACE): per-tile
# phases + per-wave lag (tools/stem_trace.py) and kernel time (tools/stem_probe.py), two rounds.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"
for r in 1 2; do for v in strace sp1 sp2; do
  export TQ_LIB_PATH=$R/term-quantization_amd/lib/libtq_hip_$v.so
  echo "== round $r $v"
  timeout -k 10 120 python tools/stem_trace.py 2>&1 | grep -v amdgpu.ids || exit 1
  timeout -k 10 120 python tools/stem_probe.py --iters 30 2>&1 | grep stem || exit 1
done; done
