#!/bin/bash
# One GPU-box check of HEAD: the given test files first (-rP prints their reports), then the
# whole -m gpu suite, smoke(), and the default bench line.  Outputs under gpurun_out/<tag>/.
# Usage: bash tools/gpu_check.sh <tag> [test files ...]
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-check}; shift || true
O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest "$@" -m gpu -x -v -rP --timeout 300 \
      --timeout-method thread > $O/first.log 2>&1
  rc=$?; tail -3 $O/first.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/first.log | head -20; exit $rc; }
fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > $O/gpu_tests.log 2>&1
rc=$?; tail -2 $O/gpu_tests.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error" $O/gpu_tests.log | head; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err
rc=$?; [ $rc -ne 0 ] && { tail -20 $O/bench.err; exit $rc; }
python3 - <<PY
import json
d = json.loads(open("$O/bench.json").read().strip().splitlines()[-1])
r = d["roofline"]
print("value %.0f img/s  ms/step %.3f  conv frac %.3f (%.1f us)  stem %.1f us" % (
    d["value"], d["ms_per_step"], r["frac"], r["avg_launch_us"], d["roofline_tr"]["avg_launch_us"]))
print("d1", json.dumps(d.get("d1_tr_op", {}))[:300])
for k, v in d.get("d4", {}).items():
    print("d4", k, {kk: vv for kk, vv in v.items() if kk in ("images_per_s", "tokens_per_s", "dominant_kernel")})
print("cpu", json.dumps(d.get("cpu_baseline", {}))[:200])
PY
