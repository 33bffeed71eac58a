#!/bin/bash
# GPU box: the three-role FVP kernel k_kz — parity / split-accuracy / sharded tests,
# then the bench (1M and the 125k shard) on k_kz and on k_kx (MJRL_AMD_FVP=kx).
# Usage (repo root, on the box): bash tools/gpu_kz.sh <tag> [pytest -k expr]
TAG=${1:-kz}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_parity.py tests/test_gpu_sharded.py -x -v --timeout 120 --timeout-method thread ${2:+-k} ${2:+"$2"} > $OUT/t.log 2>&1 \
  || { echo "TESTS FAILED"; grep -E "FAILED|Error|error|assert" $OUT/t.log | head -30; tail -5 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
for v in kz kx; do
  for a in "c4:" "p125:--paths 125"; do
    name=${a%%:*}; args=${a#*:}
    if [ $v = kx ]; then export MJRL_AMD_FVP=kx; else unset MJRL_AMD_FVP; fi
    timeout -k 10 300 python -u bench.py $args --steps 10 --warmup 3 --no-cpu-baseline --no-e2e --no-f32 > $OUT/b_${v}_$name.json 2> $OUT/b_${v}_$name.err \
      || { echo "bench $v $name failed"; tail $OUT/b_${v}_$name.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/b_${v}_$name.json'));r=d['roofline'];print('$v $name', d['ms_per_step'], d.get('hipgraph'), r['kernels'][r['kernel']]['avg_ms'], r['frac'])"
  done
done
unset MJRL_AMD_FVP
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof_c4 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --no-f32 > $GRAFT_REPO_ROOT/$OUT/prof_c4.log 2>&1 ) \
  || { echo "prof failed"; tail $OUT/prof_c4.log; exit 1; }
python tools/prof_summary.py $OUT/prof_c4 > $OUT/kernel_stats_c4.txt && head -12 $OUT/kernel_stats_c4.txt
echo KZ_DONE
