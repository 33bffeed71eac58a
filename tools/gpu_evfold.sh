#!/bin/bash
# GPU box: A/B of EVAL's first-layer fold (default: folded into P2 while loading its
# operand; variant -DMJRL_KX_EVAL_FOLD_PHASE: a phase of its own), alternating, then
# the EVAL-heavy parity tests on the default build.  Usage: bash tools/gpu_evfold.sh <tag>
OUT=gpurun_out/${1:-evfold}
mkdir -p $OUT
for r in 1 2; do
  for v in "" _evfold; do
    for T in 1000000 125000; do
      MJRL_AMD_LIB=mjrl_amd/lib/libmjrl_amd$v.so timeout -k 10 200 python -u tools/fvp_time.py $T > $OUT/t_${T}${v}_$r.txt 2>&1 || { echo "fvp_time $v $T failed"; tail $OUT/t_${T}${v}_$r.txt; exit 1; }
      echo "${v:-default} $(grep -v amdgpu.ids $OUT/t_${T}${v}_$r.txt | tail -1)"
    done
  done
done
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_split.py tests/test_gpu_fused_pack.py tests/test_gpu_sharded.py tests/test_gpu_train_step.py -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error|assert" $OUT/tests.log | head -20; exit 1; }
tail -1 $OUT/tests.log
