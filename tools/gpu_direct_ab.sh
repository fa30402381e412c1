set -u
cd ${GRAFT_REPO_ROOT:-/root/repo}
for L in 5; do for r in 1 2; do for v in default dab2 dab3 dab6 dab7; do
  lib=""; [ "$v" != default ] && lib=$PWD/term-quantization_amd/lib/libtq_hip_$v.so
  TQ_LIB_PATH=$lib timeout -k 10 120 python -u tools/conv_probe.py --layer $L --config 0 --codes 1 --no-out --nonneg --iters 30 2>/dev/null | grep layer | sed "s/^/r$r $v /" || exit 1
done; done; done
