set -u
O=gpurun_out/r06n; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_head.py tests/test_gpu_fused_parity.py tests/test_gpu_fused.py tests/test_gpu_c64.py -x -q --timeout 400 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do for v in 1 0; do
  TQ_HEAD=$v timeout -k 10 300 python3 bench.py --no-d4 --no-d1 --no-cpu-baseline --no-stem-leg > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err
  rc=$?; [ $rc -ne 0 ] && { tail -5 $O/b_${v}_$r.err; exit $rc; }
  python3 -c "import json; d=json.loads(open('$O/b_${v}_$r.json').read().strip().splitlines()[-1]); print('head=$v', round(d['value']), round(d['ms_per_step'],4), 'acc', d['accuracy_counters'])"
done; done
echo done
