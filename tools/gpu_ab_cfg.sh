#!/bin/bash
# GPU box: GPU parity tests on the default library, then per-config bench A/B of the
# default library vs MJRL_AMD_LIB=$1, for the configs in $3 (default "c3 c5").
OUT=gpurun_out/${2:-abcfg}
CFGS=${3:-"c3 c5"}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/t.log 2>&1 || { echo "TESTS FAILED"; tail -30 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
for c in $CFGS; do
  for v in default variant default variant; do
    if [ $v = variant ]; then export MJRL_AMD_LIB=$1; else unset MJRL_AMD_LIB; fi
    timeout -k 10 200 python -u bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline --no-e2e --no-f32 > $OUT/b_${c}_$v.json 2> $OUT/b_${c}_$v.err || { echo "bench $c $v failed"; tail $OUT/b_${c}_$v.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/b_${c}_$v.json'));print('$c $v', d['ms_per_step'], d.get('eager_ms_per_step'), {k: v['avg_ms'] for k, v in d['roofline']['kernels'].items()})"
  done
done
