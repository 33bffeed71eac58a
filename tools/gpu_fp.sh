#!/bin/bash
# GPU box: phase profile of k_fused on the Swimmer shape (12.5k rows and one tile).
OUT=gpurun_out/${1:-fp}
mkdir -p $OUT
export TMPDIR=/tmp
for T in 12500 64; do
MJRL_AMD_LIB=mjrl_amd/lib/libmjrl_amd_prof.so timeout -k 10 200 python -u tools/fused_prof.py $T > $OUT/fused_prof_$T.txt 2>&1 || { echo prof failed; tail $OUT/fused_prof_$T.txt; exit 1; }
cat $OUT/fused_prof_$T.txt
done
