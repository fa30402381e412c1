#!/bin/bash
# Round-2 record at HEAD: full -m gpu suite, smoke, torchrun (1 rank, RCCL + graph + chunk
# streams), then tools/gpu_profile.sh (bench JSON, kernel traces, PMC passes).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-r02_final}; O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -2 $O/gpu_tests.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error" $O/gpu_tests.log | head; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 10 --warmup 3 > $O/torchrun1.json 2> $O/torchrun1.err || { tail -20 $O/torchrun1.err; exit 1; }
python -c "import json; d=json.loads(open('$O/torchrun1.json').read().strip().splitlines()[-1]); print('torchrun n=1', round(d['value']), d['config']['launch'], d['config']['streams'])"
bash tools/gpu_profile.sh $TAG
