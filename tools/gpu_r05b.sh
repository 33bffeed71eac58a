#!/bin/bash
# Round 5: staging conversion probe, pooled update timing, pool / staging GPU tests.
OUT=gpurun_out/r05b
mkdir -p $OUT
export TMPDIR=/tmp
for pin in node0 none; do
  timeout -k 10 200 python -u tools/stage_convert_probe.py 16 $pin > $OUT/stage_probe2_$pin.txt 2>&1 || { echo "PROBE FAILED"; exit 1; }
done
timeout -k 10 300 python3 -m pytest tests/test_gpu_pool.py -x -q -p no:cacheprovider > $OUT/pytest_pool.txt 2>&1 || { echo "POOL TESTS FAILED"; tail -30 $OUT/pytest_pool.txt; exit 1; }
tail -n 1 $OUT/pytest_pool.txt
MJRL_AMD_POOL_BACKEND=gloo timeout -k 10 300 python -u tools/pool_bench.py --mode pool > $OUT/pool_pool.json 2> $OUT/pool_pool.err || { echo "POOL BENCH FAILED"; tail -20 $OUT/pool_pool.err; exit 1; }
timeout -k 10 300 python -u tools/pool_bench.py --mode local > $OUT/pool_local.json 2> $OUT/pool_local.err || { echo "LOCAL BENCH FAILED"; tail -20 $OUT/pool_local.err; exit 1; }
echo R05B_DONE
