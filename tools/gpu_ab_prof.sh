#!/bin/bash
# GPU box: parity / split tests on the default library, then rocprofv3 kernel
# stats of the default 1M bench on the default library and on a variant
# (MJRL_AMD_LIB=$1), alternating twice.  Usage: bash tools/gpu_ab_prof.sh <variant.so> <tag> [pytest -k filter]
VAR=$1; TAG=${2:-abp}; FILT=${3:-"split or parity"}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -k "$FILT" -x -q --timeout 120 --timeout-method thread > $OUT/t.log 2>&1 || { echo "TESTS FAILED"; tail -30 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
for i in 1 2; do
  for v in default variant; do
    if [ $v = variant ]; then LIBARG="MJRL_AMD_LIB=$GRAFT_REPO_ROOT/$VAR"; else LIBARG="MJRL_AMD_LIB="; fi
    ( cd /tmp && export $LIBARG && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof_${v}_$i -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --no-f32 > $GRAFT_REPO_ROOT/$OUT/prof_${v}_$i.log 2>&1 ) || { echo "prof $v failed"; tail $OUT/prof_${v}_$i.log; exit 1; }
    python tools/prof_summary.py $OUT/prof_${v}_$i > $OUT/kernel_stats_${v}_$i.txt
    echo "== $v $i $(python -c "import json;print(json.loads(open('$OUT/prof_${v}_$i.log').read().strip().splitlines()[-1])['ms_per_step'])" 2>/dev/null)"
    grep -E "k_kx|pack_split|colmax" $OUT/kernel_stats_${v}_$i.txt | cut -c1-130
  done
done
