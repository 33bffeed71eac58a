#!/bin/bash
# GPU box: k_kz vs k_kx at 1M (parity subset on the default build first), then the
# whole GPU suite once on the device-checked build (MJRL_DEVICE_CHECKS: every slab
# index against the scratch, lib/libmjrl_amd_dbg.so).
TAG=${1:-r04b}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $OUT/t.log 2>&1 \
  || { echo "TESTS FAILED"; grep -E "FAILED|Error|error|assert" $OUT/t.log | head -30; tail -5 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
for v in kz kx; do
  timeout -k 10 300 env MJRL_AMD_FVP=$v python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-e2e --no-f32 > $OUT/b_$v.json 2> $OUT/b_$v.err \
    || { echo "bench $v failed"; tail $OUT/b_$v.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/b_$v.json'));r=d['roofline'];print('$v', d['ms_per_step'], r['kernels'][r['kernel']]['avg_ms'], r['frac'])"
done
timeout -k 10 120 python -u tools/gae_probe.py > $OUT/gae_probe.txt 2>&1 && cat $OUT/gae_probe.txt || { echo gae probe failed; tail $OUT/gae_probe.txt; exit 1; }
MJRL_AMD_LIB=mjrl_amd/lib/libmjrl_amd_dbg.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/t_dbg.log 2>&1 \
  || { echo "DEBUG SUITE FAILED"; grep -E "MJRL_SLAB_CHECK|FAILED|Error|error" $OUT/t_dbg.log | head -30; tail -5 $OUT/t_dbg.log; exit 1; }
tail -1 $OUT/t_dbg.log
echo R04B_DONE
