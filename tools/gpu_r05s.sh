#!/bin/bash
# Round 5: the batch assembly fused into the forward pass (mjrl_policy_vpg_pack):
# its bit-identity tests, the split / parity / full-scale files, then bench A/B
# (MJRL_AMD_FUSED_PACK=0 vs default, alternating) at 1M and at the 125k shard.
OUT=gpurun_out/r05s
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -m pytest tests/test_gpu_fused_pack.py tests/test_gpu_split.py tests/test_gpu_parity.py tests/test_gpu_full_scale.py -x -q -p no:cacheprovider > $OUT/pytest.txt 2>&1; rc=$?
tail -3 $OUT/pytest.txt
[ $rc -eq 0 ] || { echo "TESTS FAILED rc=$rc"; grep -E "Error|assert|FAILED|Fault|fault" $OUT/pytest.txt | head -30; exit 1; }
for i in 1 2; do
  for v in 0 1; do
    MJRL_AMD_FUSED_PACK=$v timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-e2e --no-f32 > $OUT/bench_fp$v.$i.json 2> $OUT/bench_fp$v.$i.err || { echo "bench failed"; tail $OUT/bench_fp$v.$i.err; exit 1; }
    MJRL_AMD_FUSED_PACK=$v timeout -k 10 300 python -u bench.py --paths 125 --steps 10 --warmup 3 --no-cpu-baseline --no-e2e --no-f32 > $OUT/bench_p125_fp$v.$i.json 2> $OUT/bench_p125_fp$v.$i.err || { echo "bench failed"; tail $OUT/bench_p125_fp$v.$i.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/bench_fp$v.$i.json'));e=json.load(open('$OUT/bench_p125_fp$v.$i.json'));print('fused=$v', d['ms_per_step'], 'p125', e['ms_per_step'])"
  done
done
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --no-f32 > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1 ) || { echo "prof failed"; tail $OUT/prof.log; exit 1; }
python tools/prof_summary.py $OUT/prof > $OUT/kernel_stats.txt && head -8 $OUT/kernel_stats.txt
echo R05S_DONE
