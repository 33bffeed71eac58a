#!/bin/bash
# GPU box: smoke, the default bench line (full-1M CPU baseline, e2e timeline), the
# pooled 1M update (2 gloo workers on one GPU) against the in-process one, and a
# rocprofv3 kernel-trace summary of the default bench.
TAG=${1:-r04c}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH FAILED; tail -20 $OUT/bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));print('bench', d['ms_per_step'], d['vs_baseline'], d['vs_cpu_baseline'], d['cpu_baseline']['value'], d['e2e_from_host']['ms_per_step'], d['e2e_from_host']['timeline'])"
for mode in local pool; do
  MJRL_AMD_POOL_BACKEND=gloo timeout -k 10 400 python -u tools/pool_bench.py --mode $mode > $OUT/pool_$mode.json 2> $OUT/pool_$mode.err || { echo "POOL $mode FAILED"; tail -20 $OUT/pool_$mode.err; exit 1; }
  cat $OUT/pool_$mode.json
done
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --no-f32 > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1 ) \
  || { echo "prof failed"; tail $OUT/prof.log; exit 1; }
python tools/prof_summary.py $OUT/prof > $OUT/kernel_stats.txt && head -12 $OUT/kernel_stats.txt
echo R04C_DONE
