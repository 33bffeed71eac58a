#!/bin/bash
# Round 5: FVP phase ablations (timing only) + the r05b staging / pool measurements.
OUT=gpurun_out/r05c
mkdir -p $OUT
export TMPDIR=/tmp
for v in default abl_nop6 abl_nop1 abl_nochain default; do
  if [ $v = default ]; then unset MJRL_AMD_LIB; else export MJRL_AMD_LIB=mjrl_amd/lib/libmjrl_amd_$v.so; fi
  timeout -k 10 120 python -u tools/fvp_time.py 1000000 >> $OUT/ablation.txt 2>&1 || { echo "FVP TIME $v FAILED"; tail $OUT/ablation.txt; exit 1; }
  timeout -k 10 120 python -u tools/fvp_time.py 125000 >> $OUT/ablation.txt 2>&1 || { echo "FVP TIME $v FAILED"; exit 1; }
done
unset MJRL_AMD_LIB
grep -v amdgpu.ids $OUT/ablation.txt
bash tools/gpu_r05b.sh
