set -u
cd ${GRAFT_REPO_ROOT:-/root/repo}
bash tools/gpu_pmc_cmd.sh pmc_ring_def conv2d_tp_ring "python3 tools/conv_probe.py --layer 6 --config 13 --codes 1 --nonneg --residual --iters 10" > gpurun_out/pmc_ring_def.txt 2>&1
TQ_LIB_PATH=$PWD/term-quantization_amd/lib/libtq_hip_rab4.so bash tools/gpu_pmc_cmd.sh pmc_ring_ab4 conv2d_tp_ring "python3 tools/conv_probe.py --layer 6 --config 13 --codes 1 --nonneg --residual --iters 10" > gpurun_out/pmc_ring_ab4.txt 2>&1
