#!/bin/bash
# Round 5 end: per-config bench lines with CPU baselines and their kernel traces, the
# 125k shard on the sharded path, and the whole GPU suite on the device-checked build.
TAG=${1:-r05r}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
bash tools/gpu_configs.sh $TAG || exit 1
timeout -k 10 300 python -u bench.py --paths 125 --sharded-path --steps 10 --warmup 3 --no-e2e --no-cpu-baseline > $OUT/bench_p125_sharded.json 2> $OUT/bench_p125_sharded.err || { echo "sharded failed"; tail $OUT/bench_p125_sharded.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench_p125_sharded.json'));print('p125 sharded', d['ms_per_step'], d['config']['comm'])"
MJRL_AMD_LIB=mjrl_amd/lib/libmjrl_amd_dbg.so timeout -k 10 900 python3 -m pytest tests -m gpu -x -q -p no:cacheprovider > $OUT/t_dbg.log 2>&1 \
  || { echo "DEBUG SUITE FAILED"; grep -E "MJRL_SLAB_CHECK|FAILED|Error|error" $OUT/t_dbg.log | head -30; tail -5 $OUT/t_dbg.log; exit 1; }
tail -1 $OUT/t_dbg.log
echo R05R_DONE
