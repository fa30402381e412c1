# Chunk-stream schedule sweep with the default (exact) stem: lag between the streams'
# launch sequences (TQ_STREAM_LAG) and the number of chunk streams, R interleaved rounds.
set -u
O=gpurun_out/stream_sweep; mkdir -p $O
for r in $(seq 1 ${R:-2}); do
  for cfg in "0 2" "1 2" "2 2" "0 3" "0 4"; do
    set -- $cfg
    TQ_STREAM_LAG=$1 timeout -k 10 300 python3 bench.py --streams $2 --no-d4 --no-d1 --no-cpu-baseline --no-stem-leg > $O/b_$1_$2_$r.json 2> $O/b_$1_$2_$r.err
    rc=$?; [ $rc -ne 0 ] && { tail -5 $O/b_$1_$2_$r.err; exit $rc; }
    python3 -c "import json; d=json.loads(open('$O/b_$1_$2_$r.json').read().strip().splitlines()[-1]); print('lag $1 streams $2', round(d['value']), round(d['ms_per_step'],4))"
  done
done
echo done
