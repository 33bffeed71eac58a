#!/bin/bash
# rocprofv3 kernel stats of the default library vs MJRL_AMD_LIB=$1 (bench, 1M rows)
OUT=gpurun_out/${2:-pab}
mkdir -p $OUT
export TMPDIR=/tmp
for v in base new base new; do
  if [ $v = base ]; then export MJRL_AMD_LIB=$GRAFT_REPO_ROOT/$1; else unset MJRL_AMD_LIB; fi
  rm -rf $OUT/p_$v
  ( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/p_$v -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --no-f32 > $GRAFT_REPO_ROOT/$OUT/p_$v.log 2>&1 ) || { echo "prof $v failed"; exit 1; }
  echo "== $v"; python tools/prof_summary.py $OUT/p_$v | head -9 | cut -c1-60,70-
done
