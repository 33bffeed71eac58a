#!/bin/bash
# GPU box: Swimmer (c2) kernel trace and per-update timeline (span, busy, gaps).
OUT=gpurun_out/${1:-c2prof}
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config c2 --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-f32 > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1 || { echo "PROF FAILED"; tail $GRAFT_REPO_ROOT/$OUT/prof.log; exit 1; }
cd $GRAFT_REPO_ROOT
python tools/prof_summary.py $OUT/prof > $OUT/kernel_stats.txt && head -22 $OUT/kernel_stats.txt | cut -c1-150
python tools/timeline.py $OUT/prof/run_kernel_trace.csv 3 > $OUT/timeline.txt 2>&1; head -40 $OUT/timeline.txt
