#!/bin/bash
# GPU box: SQ / LDS PMC passes of the door DAPG bench (k_rows<256> + k_wgrad) and the
# HalfCheetah TRPO bench (k_rows<128> + k_wgrad_all), one pass per counter group.
OUT=gpurun_out/${1:-pmc_c5}
mkdir -p $OUT
export TMPDIR=/tmp
for c in ${CONFIGS:-c5 c3}; do
  ( cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $GRAFT_REPO_ROOT/$OUT/$c/sq -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config $c --steps 1 --warmup 0 --no-cpu-baseline --no-e2e --no-f32 > $GRAFT_REPO_ROOT/$OUT/${c}_sq.log 2>&1 ) || { echo "sq $c failed"; tail $OUT/${c}_sq.log; exit 1; }
  ( cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA --output-format csv -d $GRAFT_REPO_ROOT/$OUT/$c/lds -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config $c --steps 1 --warmup 0 --no-cpu-baseline --no-e2e --no-f32 > $GRAFT_REPO_ROOT/$OUT/${c}_lds.log 2>&1 ) || { echo "lds $c failed"; tail $OUT/${c}_lds.log; exit 1; }
  ( cd /tmp && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $GRAFT_REPO_ROOT/$OUT/$c/fetch -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config $c --steps 1 --warmup 0 --no-cpu-baseline --no-e2e --no-f32 > $GRAFT_REPO_ROOT/$OUT/${c}_fetch.log 2>&1 ) || { echo "fetch $c failed"; tail $OUT/${c}_fetch.log; exit 1; }
  ( cd /tmp && timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $GRAFT_REPO_ROOT/$OUT/$c/write -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config $c --steps 1 --warmup 0 --no-cpu-baseline --no-e2e --no-f32 > $GRAFT_REPO_ROOT/$OUT/${c}_write.log 2>&1 ) || { echo "write $c failed"; tail $OUT/${c}_write.log; exit 1; }
  python tools/pmc_summary.py $OUT/$c > $OUT/pmc_summary_$c.txt && grep -E "k_rows|k_wgrad|k_fused|k_gather|k_cgm" $OUT/pmc_summary_$c.txt | cut -c1-500
done
echo PMC_DONE
