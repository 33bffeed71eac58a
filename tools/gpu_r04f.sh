#!/bin/bash
# GPU box, round-4 evidence: per-config bench lines + kernel-trace summaries (c2, c3,
# c5, the 125k shard one-process and on the sharded path), the PMC HBM traffic passes
# of the default 1M bench (FETCH_SIZE and WRITE_SIZE in separate passes), and the
# pooled 1M update (2 gloo workers on one GPU).  Usage: bash tools/gpu_r04f.sh <tag>
TAG=${1:-r04f}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
bash tools/gpu_configs.sh $TAG || exit 1
timeout -k 10 300 python -u bench.py --paths 125 --sharded-path --steps 10 --warmup 3 --no-cpu-baseline --no-e2e --no-f32 > $OUT/bench_p125s.json 2> $OUT/bench_p125s.err || { echo "bench p125s failed"; tail $OUT/bench_p125s.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench_p125s.json'));print('p125s', d['ms_per_step'], d.get('hipgraph'), d.get('eager_ms_per_step'))"
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof_p125s -o run -- python3 $GRAFT_REPO_ROOT/bench.py --paths 125 --sharded-path --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --no-f32 > $GRAFT_REPO_ROOT/$OUT/prof_p125s.log 2>&1 ) || { echo "prof p125s failed"; tail $OUT/prof_p125s.log; exit 1; }
python tools/prof_summary.py $OUT/prof_p125s > $OUT/kernel_stats_p125s.txt
P=$OUT/pmc
mkdir -p $P
( cd /tmp && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $GRAFT_REPO_ROOT/$P/fetch -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-e2e --no-f32 > $GRAFT_REPO_ROOT/$P/fetch.log 2>&1 ) || { echo "pmc fetch failed"; tail $P/fetch.log; exit 1; }
( cd /tmp && timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $GRAFT_REPO_ROOT/$P/write -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-e2e --no-f32 > $GRAFT_REPO_ROOT/$P/write.log 2>&1 ) || { echo "pmc write failed"; tail $P/write.log; exit 1; }
python tools/pmc_summary.py $P $P/pmc_traffic.json > $P/pmc_summary.txt && grep -E "k_kx|pack_split" $P/pmc_summary.txt | cut -c1-300
for mode in local pool; do
  MJRL_AMD_POOL_BACKEND=gloo timeout -k 10 400 python -u tools/pool_bench.py --mode $mode > $OUT/pool_$mode.json 2> $OUT/pool_$mode.err || { echo "POOL $mode FAILED"; tail -20 $OUT/pool_$mode.err; exit 1; }
  cat $OUT/pool_$mode.json
done
echo R04F_DONE
