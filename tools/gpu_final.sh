#!/bin/bash
# GPU box, end-of-round evidence: full GPU tests, smoke, the default bench line,
# a kernel-trace profile of the bench, the PMC passes (HBM traffic, SQ / LDS
# counters) and the k_kx phase profile.  Usage: bash tools/gpu_final.sh <tag>
TAG=${1:-final}
bash tools/gpu_check.sh $TAG || exit 1
bash tools/profile.sh $TAG || exit 1
python tools/pmc_summary.py gpurun_out/prof_$TAG gpurun_out/prof_$TAG/pmc_traffic.json > gpurun_out/prof_$TAG/pmc_summary.txt && grep -E "k_kx|pack_split" gpurun_out/prof_$TAG/pmc_summary.txt | cut -c1-400
MJRL_AMD_LIB=mjrl_amd/lib/libmjrl_amd_prof.so timeout -k 10 200 python -u tools/kx_prof.py 1000000 > gpurun_out/$TAG/kx_phase_profile_1M.txt 2>&1 || { echo "kx_prof failed"; exit 1; }
tail -8 gpurun_out/$TAG/kx_phase_profile_1M.txt
