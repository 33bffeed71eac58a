#!/bin/bash
# GPU box: rocprofv3 kernel-trace summary of bench configs.
# Usage: bash tools/gpu_prof_cfg.sh <tag> <config>...   (c4 = the default 1M line; c2 c3 c5 p125)
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for c in "$@"; do
  case $c in
    c4) ARGS="";;
    p125) ARGS="--paths 125";;
    *) ARGS="--config $c";;
  esac
  ( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof_$c -o run -- python3 $GRAFT_REPO_ROOT/bench.py $ARGS --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --no-f32 > $GRAFT_REPO_ROOT/$OUT/prof_$c.log 2>&1 ) || { echo "prof $c failed"; tail $OUT/prof_$c.log; exit 1; }
  python tools/prof_summary.py $OUT/prof_$c > $OUT/kernel_stats_$c.txt
  head -14 $OUT/kernel_stats_$c.txt | cut -c1-130
done
