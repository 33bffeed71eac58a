#!/bin/bash
# GPU box, round 4: the sharded-path / RCCL tests and a parity subset, then the
# 125k-row shard bench on the one-process and on the sharded path (one-rank RCCL
# communicator, the update captured with its collectives), the 1M bench, and a
# rocprofv3 kernel-trace summary of the sharded 125k bench.
# Usage (repo root, on the box): bash tools/gpu_r04.sh <tag> [pytest files...]
TAG=${1:-r04}
shift
TESTS=${@:-tests/test_gpu_sharded.py tests/test_gpu_parity.py tests/test_gpu_split.py}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest $TESTS -x -v --timeout 120 --timeout-method thread > $OUT/t.log 2>&1 \
  || { echo "TESTS FAILED"; grep -E "FAILED|Error|error|assert" $OUT/t.log | head -30; tail -5 $OUT/t.log; exit 1; }
tail -2 $OUT/t.log
for v in "p125:--paths 125" "p125s:--paths 125 --sharded-path" "c4:" "c4s:--sharded-path"; do
  name=${v%%:*}; args=${v#*:}
  timeout -k 10 300 python -u bench.py $args --steps 10 --warmup 3 --no-cpu-baseline --no-e2e --no-f32 > $OUT/b_$name.json 2> $OUT/b_$name.err \
    || { echo "bench $name failed"; tail $OUT/b_$name.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/b_$name.json'));r=d['roofline'];print('$name', d['ms_per_step'], d.get('hipgraph'), d.get('eager_ms_per_step'), r['kernel'], r['kernels'][r['kernel']]['avg_ms'], r['frac'])"
done
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof_p125s -o run -- python3 $GRAFT_REPO_ROOT/bench.py --paths 125 --sharded-path --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --no-f32 > $GRAFT_REPO_ROOT/$OUT/prof_p125s.log 2>&1 ) \
  || { echo "prof failed"; tail $OUT/prof_p125s.log; exit 1; }
python tools/prof_summary.py $OUT/prof_p125s > $OUT/kernel_stats_p125s.txt && head -25 $OUT/kernel_stats_p125s.txt
echo R04_DONE
