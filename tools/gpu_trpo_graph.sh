#!/bin/bash
# GPU box: TRPO under hipGraph replay (line search on the host after the replay) —
# the replay tests, the API / parity / train-step suites, and the HalfCheetah TRPO
# bench with graphs off / auto.
OUT=gpurun_out/${1:-trpo_graph}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_api.py tests/test_gpu_parity.py tests/test_gpu_train_step.py tests/test_gpu_sharded.py tests/test_gpu_dist.py -x -q --timeout 300 --timeout-method thread > $OUT/t.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error" $OUT/t.log | head; tail -30 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
for i in 1 2; do for g in off auto; do
  timeout -k 10 300 python -u bench.py --config c3 --graph $g --steps 10 --warmup 3 --no-cpu-baseline --no-e2e > $OUT/b_${g}_$i.json 2> $OUT/b_${g}_$i.err || { echo "bench $g failed"; tail $OUT/b_${g}_$i.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/b_${g}_$i.json'));print('$g', d['ms_per_step'], d.get('hipgraph'), d.get('eager_ms_per_step'))"
done; done
