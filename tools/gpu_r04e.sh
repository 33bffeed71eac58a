#!/bin/bash
# GPU box: the one-launch CG solve (csrc/cgf.h) against the per-iteration launches
# (bit-identity tests, then the fused-path parity cases), and the Swimmer bench with
# and without it (MJRL_AMD_CG_FUSED=0), plus a kernel-trace summary of the new one.
TAG=${1:-r04e}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_cg_fused.py -x -v --timeout 120 --timeout-method thread > $OUT/t_cgf.log 2>&1 \
  || { echo "CGF TESTS FAILED"; grep -E "FAILED|Error|error|assert" $OUT/t_cgf.log | head -30; tail -5 $OUT/t_cgf.log; exit 1; }
tail -n 1 $OUT/t_cgf.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_api.py -x -q --timeout 120 --timeout-method thread > $OUT/t.log 2>&1 \
  || { echo "TESTS FAILED"; grep -E "FAILED|Error|error|assert" $OUT/t.log | head -30; tail -5 $OUT/t.log; exit 1; }
tail -n 1 $OUT/t.log
for v in 1 0; do
  MJRL_AMD_CG_FUSED=$v timeout -k 10 300 python -u bench.py --config c2 --steps 50 --warmup 5 --no-cpu-baseline --no-e2e --no-f32 > $OUT/b_c2_$v.json 2> $OUT/b_c2_$v.err \
    || { echo "bench c2 $v failed"; tail $OUT/b_c2_$v.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/b_c2_$v.json'));print('c2 fused=$v', d['ms_per_step'], d.get('hipgraph'), d.get('eager_ms_per_step'))"
done
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof_c2 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config c2 --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-f32 > $GRAFT_REPO_ROOT/$OUT/prof_c2.log 2>&1 ) \
  || { echo "prof failed"; tail $OUT/prof_c2.log; exit 1; }
python tools/prof_summary.py $OUT/prof_c2 > $OUT/kernel_stats_c2.txt && head -12 $OUT/kernel_stats_c2.txt
echo R04E_DONE
