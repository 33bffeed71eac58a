OUT=gpurun_out/${1:-split1}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_split.py -x -v --timeout 120 --timeout-method thread > $OUT/split.log 2>&1; echo "split rc=$?"; tail -15 $OUT/split.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k c4 > $OUT/parity_c4.log 2>&1; echo "parity c4 rc=$?"; tail -8 $OUT/parity_c4.log
timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e > $OUT/bench_split.json 2> $OUT/bench_split.err; echo "bench rc=$?"; cat $OUT/bench_split.json | head -c 900; echo
timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --precision f32 > $OUT/bench_f32.json 2> $OUT/bench_f32.err; echo "bench f32 rc=$?"; head -c 400 $OUT/bench_f32.json; echo
cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1; echo "prof rc=$?"; cd $GRAFT_REPO_ROOT && python tools/prof_summary.py $OUT/prof | head -14
