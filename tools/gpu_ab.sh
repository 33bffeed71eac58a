#!/bin/bash
# GPU box: split/parity tests on the default library, then the bench on the default
# library and on a variant (MJRL_AMD_LIB=$1), alternating twice
OUT=gpurun_out/${2:-ab}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $OUT/t.log 2>&1 || { echo "TESTS FAILED"; tail -20 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
for i in 1 2; do
  for v in default variant; do
    if [ $v = variant ]; then export MJRL_AMD_LIB=$1; else unset MJRL_AMD_LIB; fi
    timeout -k 10 200 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-e2e > $OUT/b_${v}_$i.json 2> $OUT/b_${v}_$i.err || { echo "bench $v failed"; tail $OUT/b_${v}_$i.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/b_${v}_$i.json'));print('$v', d['ms_per_step'], d['roofline']['kernels'])"
  done
done
