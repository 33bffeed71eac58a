#!/bin/bash
# GPU box: the whole GPU suite on the release build, the smoke, then the k_fused /
# CG-tail tests again on the device-checked build (slab bounds).
OUT=gpurun_out/${1:-final_r04h}
mkdir -p $OUT
export TMPDIR=/tmp
bash tools/gpu_suite.sh ${1:-final_r04h} || exit 1
MJRL_AMD_LIB=mjrl_amd/lib/libmjrl_amd_dbg.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_rows_shapes.py tests/test_gpu_api.py tests/test_gpu_sharded.py tests/test_gpu_train_step.py -x -q --timeout 300 --timeout-method thread > $OUT/t_dbg.log 2>&1 \
  || { echo "DEBUG SUBSET FAILED"; grep -E "FAILED|Error|error|SLAB" $OUT/t_dbg.log | head -30; tail -5 $OUT/t_dbg.log; exit 1; }
tail -n 1 $OUT/t_dbg.log
