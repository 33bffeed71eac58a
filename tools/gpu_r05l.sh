#!/bin/bash
# Round 5: one power-of-two scale per 16-row block for the dynamic operands of k_kx
# (MJRL_KX_BLOCKSCALE, lib/libmjrl_amd_bs.so) — split / parity / full-scale tests on
# it, FVP timing A/B against the per-row scales (alternating), bench lines of both.
OUT=gpurun_out/r05l
mkdir -p $OUT
export TMPDIR=/tmp
BS=mjrl_amd/lib/libmjrl_amd_bs.so
MJRL_AMD_LIB=$BS timeout -k 10 600 python3 -m pytest tests/test_gpu_split.py tests/test_gpu_parity.py tests/test_gpu_full_scale.py -q -p no:cacheprovider > $OUT/pytest_bs.txt 2>&1; rc=$?
tail -4 $OUT/pytest_bs.txt
[ $rc -eq 0 ] || { echo "TESTS rc=$rc"; grep -E "Error|assert|FAILED" $OUT/pytest_bs.txt | head -30; }
[ $rc -le 1 ] || exit 1
for v in row bs row bs; do
  if [ $v = row ]; then unset MJRL_AMD_LIB; else export MJRL_AMD_LIB=$BS; fi
  for T in 1000000 125000; do
    echo -n "$v " >> $OUT/fvp_ab.txt
    timeout -k 10 120 python -u tools/fvp_time.py $T 2>&1 | grep -v amdgpu.ids >> $OUT/fvp_ab.txt || { echo "FVP TIME FAILED"; exit 1; }
  done
done
unset MJRL_AMD_LIB
cat $OUT/fvp_ab.txt
for v in bs row; do
  if [ $v = row ]; then unset MJRL_AMD_LIB; else export MJRL_AMD_LIB=$BS; fi
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-e2e --no-f32 > $OUT/bench_$v.json 2> $OUT/bench_$v.err || { echo "bench failed"; tail $OUT/bench_$v.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/bench_$v.json'));print('$v bench', d['ms_per_step'], d['roofline']['frac'])"
done
echo R05L_DONE
