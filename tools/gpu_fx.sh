#!/bin/bash
# GPU box: k_fused change — bit-identity against the previous build, GPU parity
# subset, the phase profile, and the Swimmer bench A/B.
OUT=gpurun_out/${1:-fx}
BASE=${2:-mjrl_amd/lib/libmjrl_amd_base.so}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/fused_exact.py dump $OUT/new.npz > $OUT/dump_new.txt 2>&1 || { echo "dump new failed"; tail $OUT/dump_new.txt; exit 1; }
MJRL_AMD_LIB=$BASE timeout -k 10 200 python -u tools/fused_exact.py dump $OUT/base.npz > $OUT/dump_base.txt 2>&1 || { echo "dump base failed"; tail $OUT/dump_base.txt; exit 1; }
cat $OUT/dump_new.txt | grep shape
python tools/fused_exact.py compare $OUT/new.npz $OUT/base.npz || { echo "NOT BIT-IDENTICAL"; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_rows_shapes.py tests/test_gpu_api.py -x -q --timeout 120 --timeout-method thread > $OUT/t.log 2>&1 || { echo "TESTS FAILED"; tail -30 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
MJRL_AMD_LIB=mjrl_amd/lib/libmjrl_amd_prof.so timeout -k 10 200 python -u tools/fused_prof.py 12500 > $OUT/fused_prof_12500.txt 2>&1 || { echo prof failed; tail $OUT/fused_prof_12500.txt; exit 1; }
cat $OUT/fused_prof_12500.txt
for i in 1 2; do for v in default base; do
  if [ $v = base ]; then export MJRL_AMD_LIB=$BASE; else unset MJRL_AMD_LIB; fi
  timeout -k 10 200 python -u bench.py --config c2 --steps 20 --warmup 3 --no-cpu-baseline --no-e2e > $OUT/b_${v}_$i.json 2> $OUT/b_${v}_$i.err || { echo "bench failed"; tail $OUT/b_${v}_$i.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/b_${v}_$i.json'));r=d['roofline'];print('$v', d['ms_per_step'], r['kernel'], r['kernels'][r['kernel']]['avg_ms'])"
done; done
