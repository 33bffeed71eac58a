#!/bin/bash
# GPU box: the split / parity tests on the default library (FVP = k_kv), then the bench
# with k_kv and with k_kx's FVP (MJRL_AMD_FVP=kx), then a kernel trace of the k_kv bench.
# Usage (repo root, on the box): bash tools/gpu_kv.sh <tag> [pytest -k expr]
TAG=${1:-kv}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
MJRL_AMD_FVP=kv timeout -k 10 400 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread ${2:+-k} ${2:+"$2"} > $OUT/t.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error|error|assert" $OUT/t.log | head -30; tail -5 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
for v in kv kx; do
  MJRL_AMD_FVP=$v timeout -k 10 200 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-e2e --no-f32 > $OUT/b_$v.json 2> $OUT/b_$v.err || { echo "bench $v failed"; tail $OUT/b_$v.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/b_$v.json'));print('$v', d['ms_per_step'], d['roofline']['kernels'])"
done
if [ -f mjrl_amd/lib/libmjrl_amd_prof.so ]; then MJRL_AMD_FVP=kv MJRL_AMD_LIB=mjrl_amd/lib/libmjrl_amd_prof.so timeout -k 10 200 python -u tools/kv_prof.py > $OUT/kv_prof.txt 2>&1 || { echo kv_prof failed; tail $OUT/kv_prof.txt; exit 1; }; cat $OUT/kv_prof.txt; fi
export MJRL_AMD_FVP=kv
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-f32 > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1 || { echo "PROF FAILED"; tail -20 $GRAFT_REPO_ROOT/$OUT/prof.log; exit 1; }
cd $GRAFT_REPO_ROOT && python tools/prof_summary.py $OUT/prof > $OUT/kernel_stats.txt && head -12 $OUT/kernel_stats.txt
