#!/bin/bash
OUT=gpurun_out/c2fix
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest "tests/test_gpu_api.py::test_moments_whiten_small_equals_three_launches" tests/test_gpu_parity.py -x -q -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error|assert" $OUT/tests.log | head -20; exit 1; }
tail -1 $OUT/tests.log
for c in c2 c3; do
timeout -k 10 300 python -u bench.py --config $c --steps 20 --warmup 3 --no-e2e --no-cpu-baseline > $OUT/bench_$c.json 2> $OUT/bench_$c.err || { echo "bench failed"; tail $OUT/bench_$c.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench_$c.json'));print('$c', d['ms_per_step'], d.get('eager_ms_per_step'))"
done
