#!/bin/bash
# GPU box: per-config bench lines (c2 Swimmer NPG, c3 HalfCheetah TRPO, c5 door DAPG,
# the 125k-row Humanoid shard one-process and on the sharded code path) with a
# rocprofv3 kernel-trace summary of each.
# Usage (repo root, on the box): bash tools/gpu_configs.sh <tag>
TAG=${1:-cfg}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for c in c2 c3 c5 p125 p125s; do
  if [ $c = p125 ]; then ARGS="--paths 125"; elif [ $c = p125s ]; then ARGS="--paths 125 --sharded-path"; else ARGS="--config $c"; fi
  timeout -k 10 400 python -u bench.py $ARGS --steps 10 --warmup 3 --no-e2e > $OUT/bench_$c.json 2> $OUT/bench_$c.err || { echo "bench $c failed"; tail $OUT/bench_$c.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/bench_$c.json'));print('$c', d['ms_per_step'], d['value'], d.get('hipgraph'), d.get('eager_ms_per_step'), d['roofline']['frac'], d.get('cpu_baseline', {}).get('value'))"
  ( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof_$c -o run -- python3 $GRAFT_REPO_ROOT/bench.py $ARGS --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --no-f32 > $GRAFT_REPO_ROOT/$OUT/prof_$c.log 2>&1 ) || { echo "prof $c failed"; tail $OUT/prof_$c.log; exit 1; }
  python tools/prof_summary.py $OUT/prof_$c > $OUT/kernel_stats_$c.txt
done
echo CONFIGS_DONE
