#!/bin/bash
# Round 5: the two-kernel FVP (MJRL_AMD_FVP=split2: k_kx<.., FVP, true> writing g0, then
# k_kxg0) — split / parity / full-scale tests on it, FVP timing A/B against the fused
# kernel (alternating), a rocprofv3 kernel trace of each kernel, the bench line.
OUT=gpurun_out/r05k
mkdir -p $OUT
export TMPDIR=/tmp
MJRL_AMD_FVP=split2 timeout -k 10 600 python3 -m pytest tests/test_gpu_split.py tests/test_gpu_parity.py tests/test_gpu_full_scale.py -x -q -p no:cacheprovider > $OUT/pytest_split2.txt 2>&1; rc=$?
tail -4 $OUT/pytest_split2.txt
[ $rc -eq 0 ] || { echo "TESTS FAILED rc=$rc"; grep -E "Error|assert|FAILED" $OUT/pytest_split2.txt | head -20; exit 1; }
for v in fused split2 fused split2; do
  if [ $v = fused ]; then unset MJRL_AMD_FVP; else export MJRL_AMD_FVP=split2; fi
  for T in 1000000 125000; do
    echo -n "$v " >> $OUT/fvp_ab.txt
    timeout -k 10 120 python -u tools/fvp_time.py $T 2>&1 | grep -v amdgpu.ids >> $OUT/fvp_ab.txt || { echo "FVP TIME FAILED"; exit 1; }
  done
done
unset MJRL_AMD_FVP
cat $OUT/fvp_ab.txt
MJRL_AMD_FVP=split2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_split2 -o run -- python3 tools/fvp_time.py 1000000 > $OUT/prof_split2.log 2>&1 || { echo "rocprof failed"; tail $OUT/prof_split2.log; exit 1; }
f=$(find $OUT/prof_split2 -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && cp "$f" $OUT/kernel_stats_split2.csv && head -8 $OUT/kernel_stats_split2.csv
MJRL_AMD_FVP=split2 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-e2e --no-f32 > $OUT/bench_split2.json 2> $OUT/bench_split2.err || { echo "bench failed"; tail $OUT/bench_split2.err; exit 1; }
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-e2e --no-f32 > $OUT/bench_fused.json 2> $OUT/bench_fused.err || { echo "bench failed"; tail $OUT/bench_fused.err; exit 1; }
for v in split2 fused; do python -c "import json;d=json.load(open('$OUT/bench_$v.json'));print('$v bench', d['ms_per_step'], d['roofline']['frac'])"; done
echo R05K_DONE
