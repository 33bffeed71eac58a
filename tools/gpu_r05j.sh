#!/bin/bash
# Round 5: the P6 over observation quarters (P6Q) — split / parity / full-scale tests,
# then FVP timing A/B against the previous form (libmjrl_amd_nop6q.so), then the bench.
OUT=gpurun_out/r05j
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -m pytest tests/test_gpu_split.py tests/test_gpu_parity.py tests/test_gpu_full_scale.py -x -q -p no:cacheprovider > $OUT/pytest.txt 2>&1; rc=$?
tail -4 $OUT/pytest.txt
[ $rc -eq 0 ] || { echo "TESTS FAILED rc=$rc"; grep -E "Error|assert|FAILED" $OUT/pytest.txt | head -20; exit 1; }
for v in default nop6q default nop6q; do
  if [ $v = default ]; then unset MJRL_AMD_LIB; else export MJRL_AMD_LIB=mjrl_amd/lib/libmjrl_amd_$v.so; fi
  timeout -k 10 120 python -u tools/fvp_time.py 1000000 2>&1 | grep -v amdgpu.ids >> $OUT/fvp_ab.txt || { echo "FVP TIME FAILED"; exit 1; }
  timeout -k 10 120 python -u tools/fvp_time.py 125000 2>&1 | grep -v amdgpu.ids >> $OUT/fvp_ab.txt || { echo "FVP TIME FAILED"; exit 1; }
done
unset MJRL_AMD_LIB
cat $OUT/fvp_ab.txt
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-e2e --no-f32 > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail $OUT/bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));print('bench', d['ms_per_step'], d['roofline']['frac'], d['roofline']['kernels'])"
echo R05G_DONE
