#!/bin/bash
# Profiles bench.py on the GPU box: kernel trace + stats, then PMC passes
# (FETCH_SIZE and WRITE_SIZE in separate passes, then SQ timing / LDS counters).
# Usage (from the repo root, on the box): bash tools/profile.sh <tag> [bench args...]
set -eo pipefail
TAG=${1:-r01}; shift || true
ARGS=${@:-"--steps 2 --warmup 1 --no-cpu-baseline --no-e2e"}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-e2e > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-e2e > $OUT/write.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-e2e > $OUT/sq.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA --output-format csv -d $OUT/lds -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-e2e > $OUT/lds.log 2>&1 || echo "lds pass failed (counter names?)"
echo PROFILE_DONE
