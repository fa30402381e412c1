#!/bin/bash
# Ring-engine phase-shift probe (RING_AB=12 build): workgroups with one tile fewer, every other
# one, start TQ_AB x ~3.4 us late.  Usage: bash tools/gpu_ring_phase.sh "<layers>" "<delays>"
# (RING_AB=12 was a timing-only build option, reverted after this probe: profiles/r05_ring_epilogue_probes.txt)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; LAYERS=$1; DELAYS=$2
for L in $LAYERS; do
  for F in "--no-out" "--residual"; do
    timeout -k 10 120 python -u tools/conv_probe.py --layer $L --config 13 --codes 1 --nonneg $F --iters 30 2>/dev/null | grep layer | sed "s/^/$F default /" || exit 1
    for d in $DELAYS; do
      TQ_AB=$d TQ_LIB_PATH=$R/term-quantization_amd/lib/libtq_hip_rab12.so timeout -k 10 120 python -u tools/conv_probe.py --layer $L --config 13 --codes 1 --nonneg $F --iters 30 2>/dev/null | grep layer | sed "s/^/$F delay$d /" || exit 1
    done
  done
done
