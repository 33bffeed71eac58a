#!/bin/bash
# GPU box: split-path tests, c4 parity, bench (split / first-layer-only split / f32), kernel-trace profile
OUT=gpurun_out/${1:-split1}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_split.py -x -v --timeout 120 --timeout-method thread > $OUT/split.log 2>&1; rc=$?; echo "split rc=$rc"; grep -E "PASS|FAIL|Error|assert" $OUT/split.log | head -20; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k c4 > $OUT/parity_c4.log 2>&1; rc=$?; echo "parity c4 rc=$rc"; grep -E "PASS|FAIL|Error|assert" $OUT/parity_c4.log | head; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e > $OUT/bench_split.json 2> $OUT/bench_split.err || { echo "bench failed"; tail $OUT/bench_split.err; exit 1; }
head -c 330 $OUT/bench_split.json; echo
MJRL_AMD_SPLIT_LAYERS=1 timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e > $OUT/bench_split1.json 2> $OUT/bench_split1.err; echo "bench split1 rc=$?"; head -c 330 $OUT/bench_split1.json; echo
cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1; echo "prof rc=$?"; cd $GRAFT_REPO_ROOT && python tools/prof_summary.py $OUT/prof | head -12
