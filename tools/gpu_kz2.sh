#!/bin/bash
# GPU box: k_kz parity subset, its interval profile (profiling build), bench k_kz vs k_kx at 1M.
TAG=${1:-kz2}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $OUT/t.log 2>&1 \
  || { echo "TESTS FAILED"; grep -E "FAILED|Error|error|assert" $OUT/t.log | head -30; tail -5 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
MJRL_AMD_LIB=mjrl_amd/lib/libmjrl_amd_prof.so timeout -k 10 200 python -u tools/kz_prof.py > $OUT/kz_prof.txt 2>&1 || { echo prof failed; tail $OUT/kz_prof.txt; exit 1; }
tail -6 $OUT/kz_prof.txt
for v in kz kx; do
  if [ $v = kx ]; then export MJRL_AMD_FVP=kx; else unset MJRL_AMD_FVP; fi
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-e2e --no-f32 > $OUT/b_$v.json 2> $OUT/b_$v.err \
    || { echo "bench $v failed"; tail $OUT/b_$v.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/b_$v.json'));r=d['roofline'];print('$v', d['ms_per_step'], r['kernels'][r['kernel']]['avg_ms'], r['frac'])"
done
echo KZ2_DONE
