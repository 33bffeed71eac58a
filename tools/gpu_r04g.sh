#!/bin/bash
# GPU box: k_kx slab writes staged through LDS — parity, the phase profile's tail at
# 125k rows, the 1M / 125k / sharded benches; then the N > 1 bench path rehearsed
# with two gloo ranks on one GPU.
TAG=${1:-r04g}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_parity.py tests/test_gpu_sharded.py -x -q --timeout 120 --timeout-method thread > $OUT/t.log 2>&1 \
  || { echo "TESTS FAILED"; grep -E "FAILED|Error|error|assert" $OUT/t.log | head -30; tail -5 $OUT/t.log; exit 1; }
tail -n 1 $OUT/t.log
MJRL_AMD_LIB=mjrl_amd/lib/libmjrl_amd_prof.so timeout -k 10 200 python -u tools/kx_prof.py 125000 > $OUT/kx_prof_125k.txt 2>&1 || { echo prof failed; tail $OUT/kx_prof_125k.txt; exit 1; }
grep -E "FVP \+|preamble|^tail|tile loop" $OUT/kx_prof_125k.txt
for c in "c4:" "p125:--paths 125" "p125s:--paths 125 --sharded-path"; do
  name=${c%%:*}; args=${c#*:}
  timeout -k 10 300 python -u bench.py $args --steps 10 --warmup 3 --no-cpu-baseline --no-e2e --no-f32 > $OUT/b_$name.json 2> $OUT/b_$name.err \
    || { echo "bench $name failed"; tail $OUT/b_$name.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/b_$name.json'));r=d['roofline'];print('$name', d['ms_per_step'], r['kernels'][r['kernel']]['avg_ms'], r['frac'])"
done
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --backend gloo --steps 3 --warmup 1 > $OUT/b_gloo2.json 2> $OUT/b_gloo2.err \
  || { echo "gloo2 bench failed"; tail -20 $OUT/b_gloo2.err; exit 1; }
cat $OUT/b_gloo2.json | cut -c1-400
echo R04G_DONE
