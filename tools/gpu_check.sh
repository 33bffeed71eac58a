#!/bin/bash
# GPU box: parity tests, then the default bench line (N=1), then a kernel-trace profile.
# Usage (repo root, on the box): bash tools/gpu_check.sh <tag>
TAG=${1:-chk}
OUT=gpurun_out/$TAG
mkdir -p $OUT
# the driver's exact command
timeout -k 10 1000 python3 -m pytest tests/ -x -q -m gpu -p no:cacheprovider > $OUT/pytest.log 2>&1 || { echo "PYTEST FAILED"; tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "SMOKE FAILED"; cat $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "BENCH FAILED"; tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1 || { echo "PROF FAILED"; tail -30 $GRAFT_REPO_ROOT/$OUT/prof.log; exit 1; }
cd $GRAFT_REPO_ROOT && python tools/prof_summary.py $OUT/prof > $OUT/kernel_stats.txt && head -25 $OUT/kernel_stats.txt
