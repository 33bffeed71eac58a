#!/bin/bash
# GPU box, end-of-round evidence at HEAD: the default bench line (full-1M CPU
# baseline, e2e timeline), a kernel-trace profile and the PMC passes of it, the k_kx
# phase profile, per-config lines with their kernel-trace summaries, the sharded
# 125k line.  Usage: bash tools/gpu_r04i.sh <tag>
TAG=${1:-r04i}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "BENCH FAILED"; tail -30 $OUT/bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));print('c4', d['ms_per_step'], d['value'], d['roofline']['frac'], d['cpu_baseline']['value'], d.get('vs_baseline'))"
bash tools/profile.sh $TAG || { echo "PROFILE FAILED"; exit 1; }
python tools/prof_summary.py gpurun_out/prof_$TAG/trace > $OUT/kernel_stats.txt && head -6 $OUT/kernel_stats.txt | cut -c1-120
python tools/pmc_summary.py gpurun_out/prof_$TAG gpurun_out/prof_$TAG/pmc_traffic.json > gpurun_out/prof_$TAG/pmc_summary.txt && grep -E "k_kx" gpurun_out/prof_$TAG/pmc_summary.txt | cut -c1-300
MJRL_AMD_LIB=mjrl_amd/lib/libmjrl_amd_prof.so timeout -k 10 200 python -u tools/kx_prof.py 1000000 > $OUT/kx_phase_profile_1M.txt 2>&1 || { echo "kx_prof failed"; exit 1; }
bash tools/gpu_configs.sh $TAG || exit 1
timeout -k 10 300 python -u bench.py --paths 125 --sharded-path --steps 10 --warmup 3 --no-cpu-baseline --no-e2e --no-f32 > $OUT/bench_p125s.json 2> $OUT/bench_p125s.err || { echo "bench p125s failed"; tail $OUT/bench_p125s.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench_p125s.json'));print('p125s', d['ms_per_step'])"
echo R04I_DONE
