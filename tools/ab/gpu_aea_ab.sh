# act_encode_act A/B: in-tree build vs lib/libtq_hip_aea1.so (the option under test off: first
# AEA_UNROLL, then AEA_NT): the tests that run it, then interleaved bench runs
# for the D4 executors (MobileNet-V2, EfficientNet-b0) and the headline.
set -u
O=gpurun_out/aea_ab; mkdir -p $O
OLD=$PWD/term-quantization_amd/lib/libtq_hip_aea1.so
timeout -k 10 600 python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do for v in new old; do
  L=$PWD/term-quantization_amd/lib/libtq_hip.so; [ $v = old ] && L=$OLD
  TQ_LIB_PATH=$L timeout -k 10 400 python3 bench.py --no-d1 --no-cpu-baseline --no-stem-leg > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err
  rc=$?; [ $rc -ne 0 ] && { tail -5 $O/b_${v}_$r.err; exit $rc; }
  python3 -c "
import json; d=json.loads(open('$O/b_${v}_$r.json').read().strip().splitlines()[-1]); d4=d['d4']
m=d4['mobilenet_v2']; e=d4['efficientnet_b0']
print('$v', 'resnet', round(d['value']), 'mbv2', round(m['images_per_s']), 'aea', round(m['kernels']['act_encode_act']['avg_launch_us'],1), round(m['kernels']['act_encode_act']['frac'],3), 'effnet', round(e['images_per_s']), 'aea', round(e['kernels']['act_encode_act']['avg_launch_us'],1), round(e['kernels']['act_encode_act']['frac'],3))"
done; done
echo done
