#!/bin/bash
# GPU box: parity of the pipelined k_kx FVP (MJRL_KX_P1PIPE) and of the GAE chain
# change, the 1M and 125k benches against the unpipelined build (libmjrl_amd_nopipe),
# the GAE probe, then the whole GPU suite on the device-checked build.
TAG=${1:-r04d}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_parity.py tests/test_gpu_api.py -x -q --timeout 120 --timeout-method thread > $OUT/t.log 2>&1 \
  || { echo "TESTS FAILED"; grep -E "FAILED|Error|error|assert" $OUT/t.log | head -30; tail -5 $OUT/t.log; exit 1; }
tail -n 1 $OUT/t.log
for v in pipe nopipe; do
  L=mjrl_amd/lib/libmjrl_amd.so; [ $v = nopipe ] && L=mjrl_amd/lib/libmjrl_amd_nopipe.so
  for c in "c4:" "p125:--paths 125"; do
    name=${c%%:*}; args=${c#*:}
    MJRL_AMD_LIB=$L timeout -k 10 300 python -u bench.py $args --steps 10 --warmup 3 --no-cpu-baseline --no-e2e --no-f32 > $OUT/b_${v}_$name.json 2> $OUT/b_${v}_$name.err \
      || { echo "bench $v $name failed"; tail $OUT/b_${v}_$name.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/b_${v}_$name.json'));r=d['roofline'];print('$v $name', d['ms_per_step'], r['kernels'][r['kernel']]['avg_ms'], r['frac'])"
  done
done
timeout -k 10 120 python -u tools/gae_probe.py > $OUT/gae_probe.txt 2>&1 && cat $OUT/gae_probe.txt || { echo gae probe failed; tail $OUT/gae_probe.txt; exit 1; }
MJRL_AMD_LIB=mjrl_amd/lib/libmjrl_amd_dbg.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/t_dbg.log 2>&1 \
  || { echo "DEBUG SUITE FAILED"; grep -E "MJRL_SLAB_CHECK|FAILED|Error|error" $OUT/t_dbg.log | head -30; tail -5 $OUT/t_dbg.log; exit 1; }
tail -n 1 $OUT/t_dbg.log
echo R04D_DONE
