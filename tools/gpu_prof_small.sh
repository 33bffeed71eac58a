#!/bin/bash
# GPU box: k_kx phase profile (profiling build) at 1M and 125k rows, plus the bench at 125k rows
OUT=gpurun_out/${1:-kxs}
mkdir -p $OUT
MJRL_AMD_LIB=mjrl_amd/lib/libmjrl_amd_prof.so timeout -k 10 200 python -u tools/kx_prof.py 1000000 > $OUT/kx_1M.txt 2>&1 || { echo "prof 1M failed"; tail $OUT/kx_1M.txt; exit 1; }
MJRL_AMD_LIB=mjrl_amd/lib/libmjrl_amd_prof.so timeout -k 10 200 python -u tools/kx_prof.py 125000 > $OUT/kx_125k.txt 2>&1 || { echo "prof 125k failed"; tail $OUT/kx_125k.txt; exit 1; }
cat $OUT/kx_1M.txt $OUT/kx_125k.txt
timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --paths 125 --no-cpu-baseline --no-e2e > $OUT/bench_125.json 2> $OUT/bench_125.err || { echo "bench failed"; tail $OUT/bench_125.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench_125.json'));print(125, d['ms_per_step'], d['value'])"
timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e > $OUT/bench_1M.json 2> $OUT/bench_1M.err || { echo "bench failed"; tail $OUT/bench_1M.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench_1M.json'));print(1000, d['ms_per_step'], d['value'])"
