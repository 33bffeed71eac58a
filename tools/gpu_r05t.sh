#!/bin/bash
# Round 5: fused-pack publish with the DPP row max: bit-identity tests, bench at 1M
# and 125k (twice), kernel trace.
OUT=gpurun_out/r05t
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -m pytest tests/test_gpu_fused_pack.py tests/test_gpu_split.py -x -q -p no:cacheprovider > $OUT/pytest.txt 2>&1; rc=$?
tail -2 $OUT/pytest.txt
[ $rc -eq 0 ] || { echo "TESTS FAILED rc=$rc"; grep -E "Error|assert|FAILED|fault" $OUT/pytest.txt | head -30; exit 1; }
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-e2e --no-f32 > $OUT/bench.$i.json 2> $OUT/bench.$i.err || { echo "bench failed"; tail $OUT/bench.$i.err; exit 1; }
  timeout -k 10 300 python -u bench.py --paths 125 --steps 10 --warmup 3 --no-cpu-baseline --no-e2e --no-f32 > $OUT/bench_p125.$i.json 2> $OUT/bench_p125.$i.err || { echo "bench failed"; tail $OUT/bench_p125.$i.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/bench.$i.json'));e=json.load(open('$OUT/bench_p125.$i.json'));print(d['ms_per_step'], 'p125', e['ms_per_step'])"
done
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --no-f32 > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1 ) || { echo "prof failed"; tail $OUT/prof.log; exit 1; }
python tools/prof_summary.py $OUT/prof > $OUT/kernel_stats.txt && head -8 $OUT/kernel_stats.txt
echo R05T_DONE
