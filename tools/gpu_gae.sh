#!/bin/bash
OUT=gpurun_out/${1:-gae}
mkdir -p $OUT
timeout -k 10 120 python3 -u tools/gae_probe.py > $OUT/gae_probe.txt 2>&1 || { echo "GAE_PROBE FAILED"; tail $OUT/gae_probe.txt; exit 1; }
cat $OUT/gae_probe.txt
timeout -k 10 300 python3 -u -m pytest "tests/test_gpu_api.py::test_gae_kernel_ragged_many_paths" "tests/test_gpu_api.py::test_gae_kernel_multiwindow_bitexact" tests/test_gpu_train_step.py "tests/test_gpu_sharded.py::test_trpo_device_line_search_equals_host" -x -q -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/gae_tests.log 2>&1 || { echo "GAE TESTS FAILED"; grep -E "FAIL|Error|assert" $OUT/gae_tests.log | head -20; exit 1; }
tail -1 $OUT/gae_tests.log
