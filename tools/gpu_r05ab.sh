#!/bin/bash
# Round 5: the fused pack's conversion moved from the publish to the end of the previous
# tile's gW0 sums (libmjrl_amd_p6pack.so): bit-identity tests on it, bench A/B alternating.
OUT=gpurun_out/r05ab
mkdir -p $OUT
export TMPDIR=/tmp
V=mjrl_amd/lib/libmjrl_amd_p6pack.so
MJRL_AMD_LIB=$V timeout -k 10 400 python3 -m pytest tests/test_gpu_fused_pack.py tests/test_gpu_split.py -x -q -p no:cacheprovider > $OUT/pytest.txt 2>&1; rc=$?
tail -2 $OUT/pytest.txt
[ $rc -eq 0 ] || { echo "TESTS FAILED rc=$rc"; grep -E "Error|assert|FAILED|fault" $OUT/pytest.txt | head -20; exit 1; }
for i in 1 2; do
  for v in pub p6; do
    if [ $v = pub ]; then unset MJRL_AMD_LIB; else export MJRL_AMD_LIB=$V; fi
    timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-e2e --no-f32 > $OUT/bench_$v.$i.json 2> $OUT/bench_$v.$i.err || { echo "bench failed"; tail $OUT/bench_$v.$i.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/bench_$v.$i.json'));print('$v', d['ms_per_step'])"
  done
done
unset MJRL_AMD_LIB
for v in pub p6; do
  if [ $v = pub ]; then unset MJRL_AMD_LIB; else export MJRL_AMD_LIB=$V; fi
  ( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof_$v -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --no-f32 > $GRAFT_REPO_ROOT/$OUT/prof_$v.log 2>&1 ) || { echo "prof failed"; exit 1; }
  python tools/prof_summary.py $OUT/prof_$v | grep "k_kx<32, 12, 0"
done
echo R05AB_DONE
