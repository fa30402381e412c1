set -u
cd ${GRAFT_REPO_ROOT:-/root/repo}
for r in 1 2; do
for s in 1 2 4; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-d1 --no-d4 --no-stem-leg --streams $s 2>/dev/null | python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('round $r streams $s', round(d['value']), round(d['ms_per_step'],3))" || exit 1
done
done
