set -u
O=gpurun_out/r06o; mkdir -p $O
L2=$PWD/term-quantization_amd/lib/libtq_hip_epif32.so
TQ_LIB_PATH=$L2 timeout -k 10 900 python -u -m pytest tests/test_gpu_fused_parity.py tests/test_gpu_c64.py tests/test_gpu_ring.py -x -q --timeout 400 --timeout-method thread > $O/tests_epif32.log 2>&1
rc=$?; tail -2 $O/tests_epif32.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2 3; do for v in base epif32; do
  L=$PWD/term-quantization_amd/lib/libtq_hip.so; [ $v != base ] && L=$L2
  TQ_LIB_PATH=$L timeout -k 10 300 python3 bench.py --no-d4 --no-d1 --no-cpu-baseline --no-stem-leg > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err
  rc=$?; [ $rc -ne 0 ] && { tail -5 $O/b_${v}_$r.err; exit $rc; }
  python3 -c "import json; d=json.loads(open('$O/b_${v}_$r.json').read().strip().splitlines()[-1]); print('$v', round(d['value']), round(d['ms_per_step'],4), 'conv', round(d['roofline']['avg_launch_us'],2), 'stem', round(d['roofline_tr']['avg_launch_us'],1))"
done; done
echo done
