#!/bin/bash
# Round 6, end-of-round evidence part 2 (after tools/gpu_check.sh): the PMC passes of
# the default bench (HBM traffic, SQ / LDS counters) and their summary, the k_kx phase
# profile, then every config's bench line and kernel trace.  Usage: bash tools/gpu_r06d.sh <tag>
TAG=${1:-r06d}
bash tools/profile.sh $TAG || { echo "PROFILE FAILED"; exit 1; }
python tools/pmc_summary.py gpurun_out/prof_$TAG gpurun_out/prof_$TAG/pmc_traffic.json > gpurun_out/prof_$TAG/pmc_summary.txt && grep -E "k_kx|k_gae" gpurun_out/prof_$TAG/pmc_summary.txt | cut -c1-300
mkdir -p gpurun_out/$TAG
MJRL_AMD_LIB=mjrl_amd/lib/libmjrl_amd_prof.so timeout -k 10 200 python -u tools/kx_prof.py 1000000 > gpurun_out/$TAG/kx_phase_profile_1M.txt 2>&1 || { echo "kx_prof failed"; exit 1; }
tail -4 gpurun_out/$TAG/kx_phase_profile_1M.txt
bash tools/gpu_configs.sh $TAG/cfg || exit 1
