#!/bin/bash
# GPU box: the bench line and a rocprofv3 kernel trace of the SAME command, for the
# roofline's launch duration against the profiler's average.  Usage: bash tools/gpu_pair.sh <tag>
TAG=${1:-pair}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--steps 10 --warmup 3 --no-cpu-baseline --no-e2e --no-f32"
timeout -k 10 300 python -u bench.py $ARGS > $OUT/bench.json 2> $OUT/bench.err || { echo "BENCH FAILED"; tail $OUT/bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));r=d['roofline'];print('bench', d['ms_per_step'], r['kernels'][r['kernel']]['avg_ms'], r['frac'], r.get('traffic_source'))"
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py $ARGS > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1 ) || { echo "PROF FAILED"; tail $OUT/prof.log; exit 1; }
python tools/prof_summary.py $OUT/prof > $OUT/kernel_stats.txt && head -6 $OUT/kernel_stats.txt | cut -c1-120
grep -h '"ms_per_step"' $OUT/prof.log | head -1 | cut -c1-200
