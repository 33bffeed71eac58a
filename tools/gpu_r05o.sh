#!/bin/bash
# Round 5: pool fill with two chunks per controller thread and the native 1-D gather:
# pool GPU tests, pooled vs in-process update timing.
OUT=gpurun_out/r05o
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -m pytest tests/test_gpu_pool.py -x -q -p no:cacheprovider > $OUT/pytest_pool.txt 2>&1 || { echo "POOL TESTS FAILED"; tail -30 $OUT/pytest_pool.txt; exit 1; }
tail -n 1 $OUT/pytest_pool.txt
MJRL_AMD_POOL_BACKEND=gloo timeout -k 10 300 python -u tools/pool_bench.py --mode pool > $OUT/pool_pool.json 2> $OUT/pool_pool.err || { echo "POOL BENCH FAILED"; tail -20 $OUT/pool_pool.err; exit 1; }
timeout -k 10 300 python -u tools/pool_bench.py --mode local > $OUT/pool_local.json 2> $OUT/pool_local.err || { echo "LOCAL BENCH FAILED"; tail -20 $OUT/pool_local.err; exit 1; }
grep -h ms_per_update $OUT/pool_pool.json $OUT/pool_local.json | cut -c1-700
echo R05O_DONE
