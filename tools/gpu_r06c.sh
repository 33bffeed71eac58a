#!/bin/bash
# Round 6, GPU pass c: the GAE probe, the GAE tests then the whole GPU suite + smoke,
# the default bench line (with its CPU baseline), the per-config lines.
TAG=${1:-r06c}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 python3 -u tools/gae_probe.py > $OUT/gae_probe.txt 2>&1 || { echo "GAE_PROBE FAILED"; tail $OUT/gae_probe.txt; exit 1; }
cat $OUT/gae_probe.txt
timeout -k 10 300 python3 -u -m pytest "tests/test_gpu_api.py::test_gae_kernel_ragged_many_paths" "tests/test_gpu_api.py::test_gae_kernel_multiwindow_bitexact" "tests/test_gpu_api.py::test_moments_whiten_small_equals_three_launches" tests/test_gpu_stream_staging.py tests/test_gpu_sharded.py tests/test_gpu_train_step.py -x -q -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/gae_tests.log 2>&1 || { echo "GAE TESTS FAILED"; grep -E "FAIL|Error|assert" $OUT/gae_tests.log | head -20; exit 1; }
tail -1 $OUT/gae_tests.log
bash tools/gpu_suite.sh $TAG/suite || exit 1
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "BENCH FAILED"; tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
bash tools/gpu_configs.sh $TAG/cfg || exit 1
