#!/bin/bash
# GPU box: A/B of an environment switch on bench lines.
# Usage: bash tools/gpu_env_ab.sh <tag> <VAR> <value_a> <value_b> [pytest -k filter] [bench configs...]
# Runs the GPU tests matching the filter (if given) first, then for each config
# (c4 = the default 1M Humanoid line, c2 / c3 / c5 / p125) the bench with VAR=a
# and VAR=b, alternating twice.
TAG=$1; VAR=$2; A=$3; B=$4; FILT=$5; shift 5
CFGS=${@:-c4}
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ -n "$FILT" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -k "$FILT" -x -q --timeout 120 --timeout-method thread > $OUT/t.log 2>&1 || { echo "TESTS FAILED"; tail -30 $OUT/t.log; exit 1; }
  tail -1 $OUT/t.log
fi
for c in $CFGS; do
  case $c in
    c4) ARGS="";;
    p125) ARGS="--paths 125";;
    *) ARGS="--config $c";;
  esac
  for i in 1 2; do
    for val in $A $B; do
      env $VAR=$val timeout -k 10 200 python -u bench.py $ARGS --steps 10 --warmup 3 --no-cpu-baseline --no-e2e --no-f32 > $OUT/b_${c}_${val}_$i.json 2> $OUT/b_${c}_${val}_$i.err || { echo "bench $c $val failed"; tail $OUT/b_${c}_${val}_$i.err; exit 1; }
      python -c "import json;d=json.load(open('$OUT/b_${c}_${val}_$i.json'));print('$c $VAR=$val', d['ms_per_step'], d.get('hipgraph'), d.get('eager_ms_per_step'))"
    done
  done
done
