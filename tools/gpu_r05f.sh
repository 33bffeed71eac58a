#!/bin/bash
# Round 5: k_rows FVP on split-f16 products — rows-shape fp64 tests, C3 / C5 parity, per-config bench lines.
OUT=gpurun_out/r05f
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -m pytest tests/test_gpu_rows_shapes.py "tests/test_gpu_parity.py" -x -q -p no:cacheprovider -k "rows or c3 or c5" > $OUT/pytest.txt 2>&1; rc=$?
tail -15 $OUT/pytest.txt
[ $rc -eq 0 ] || { echo "TESTS FAILED rc=$rc"; exit 1; }
for c in c3 c5; do
  timeout -k 10 300 python -u bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline --no-e2e > $OUT/bench_$c.json 2> $OUT/bench_$c.err || { echo "bench $c failed"; tail $OUT/bench_$c.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/bench_$c.json'));print('$c', d['ms_per_step'], d['dtype'], d.get('f32_ms_per_step'), d['roofline']['kernels'])"
done
echo R05F_DONE
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof_c3 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config c3 --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --no-f32 > $GRAFT_REPO_ROOT/$OUT/prof_c3.log 2>&1 || { echo "PROF FAILED"; exit 1; }
cd $GRAFT_REPO_ROOT && python tools/prof_summary.py $OUT/prof_c3 > $OUT/kernel_stats_c3.txt && head -12 $OUT/kernel_stats_c3.txt
