#!/bin/bash
# Round 5: k_wgrad with 128 x 128 output blocks for the square job — rows-shape / C5 tests, door bench + rocprof.
OUT=gpurun_out/r05i
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -m pytest tests/test_gpu_rows_shapes.py tests/test_gpu_parity.py -x -q -p no:cacheprovider -k "rows or c5" > $OUT/pytest.txt 2>&1; rc=$?
tail -3 $OUT/pytest.txt
[ $rc -eq 0 ] || { echo "TESTS FAILED rc=$rc"; grep -E "Error|assert|FAILED" $OUT/pytest.txt | head -20; exit 1; }
timeout -k 10 300 python -u bench.py --config c5 --steps 10 --warmup 3 --no-cpu-baseline --no-e2e > $OUT/bench_c5.json 2> $OUT/bench_c5.err || { echo "bench failed"; tail $OUT/bench_c5.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench_c5.json'));print('c5', d['ms_per_step'], d['roofline']['kernels'])"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof_c5 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline --no-e2e > $GRAFT_REPO_ROOT/$OUT/prof_c5.log 2>&1 || { echo "PROF FAILED"; exit 1; }
cd $GRAFT_REPO_ROOT && python tools/prof_summary.py $OUT/prof_c5 > $OUT/kernel_stats_c5.txt && head -8 $OUT/kernel_stats_c5.txt
echo R05I_DONE
