#!/bin/bash
# Round 6, GPU pass b: GAE microbenchmarks, the new / changed parity tests, the
# whole GPU suite + smoke, the bench line, the PMC passes at this commit.
TAG=${1:-r06b}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 60 ./tools/gae_latency > $OUT/gae_latency.txt 2>&1 || { echo "GAE_LATENCY FAILED"; cat $OUT/gae_latency.txt; exit 1; }
cat $OUT/gae_latency.txt
timeout -k 10 120 python3 -u tools/gae_probe.py > $OUT/gae_probe.txt 2>&1 || { echo "GAE_PROBE FAILED"; tail $OUT/gae_probe.txt; exit 1; }
cat $OUT/gae_probe.txt
timeout -k 10 400 python3 -u -m pytest "tests/test_gpu_api.py::test_gae_kernel_ragged_many_paths" "tests/test_gpu_api.py::test_gae_kernel_multiwindow_bitexact" tests/test_gpu_f64obs.py tests/test_gpu_stream_staging.py tests/test_gpu_train_step.py tests/test_gpu_sharded.py -x -v -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/new_tests.log 2>&1 || { echo "NEW TESTS FAILED"; grep -E "PASS|FAIL|Error" $OUT/new_tests.log | tail -40; exit 1; }
grep -cE "PASSED" $OUT/new_tests.log
bash tools/gpu_suite.sh $TAG/suite || exit 1
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { echo "BENCH FAILED"; tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
bash tools/profile.sh $TAG || exit 1
python tools/pmc_summary.py gpurun_out/prof_$TAG gpurun_out/prof_$TAG/pmc_traffic.json > gpurun_out/prof_$TAG/pmc_summary.txt && grep -E "k_kx" gpurun_out/prof_$TAG/pmc_summary.txt | cut -c1-300
python tools/prof_summary.py gpurun_out/prof_$TAG/trace > gpurun_out/prof_$TAG/kernel_stats.txt && head -12 gpurun_out/prof_$TAG/kernel_stats.txt
