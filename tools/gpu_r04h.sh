#!/bin/bash
# GPU box: CG tail loads issued up front (k_cgm_xrp_f, the flat gather's z step) —
# bit-identity against the previous build, GPU tests, per-config benches and a
# rocprof summary of the Swimmer update.
OUT=gpurun_out/${1:-r04h}
BASE=${2:-mjrl_amd/lib/libmjrl_amd_base.so}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/fused_exact.py dump $OUT/new.npz > $OUT/dump_new.txt 2>&1 || { echo "dump new failed"; tail -20 $OUT/dump_new.txt; exit 1; }
MJRL_AMD_LIB=$BASE timeout -k 10 300 python -u tools/fused_exact.py dump $OUT/base.npz > $OUT/dump_base.txt 2>&1 || { echo "dump base failed"; tail $OUT/dump_base.txt; exit 1; }
python tools/fused_exact.py compare $OUT/new.npz $OUT/base.npz || { echo "NOT BIT-IDENTICAL"; exit 1; }
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sharded.py tests/test_gpu_split.py tests/test_gpu_rows_shapes.py tests/test_gpu_api.py -x -q --timeout 120 --timeout-method thread > $OUT/t.log 2>&1 || { echo "TESTS FAILED"; tail -30 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
for c in "c2:--config c2" "c2b:--config c2" "p125:--paths 125" "p125s:--paths 125 --sharded-path" "c4:"; do
  name=${c%%:*}; args=${c#*:}
  timeout -k 10 300 python -u bench.py $args --steps 10 --warmup 3 --no-cpu-baseline --no-e2e --no-f32 > $OUT/b_$name.json 2> $OUT/b_$name.err \
    || { echo "bench $name failed"; tail $OUT/b_$name.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/b_$name.json'));r=d['roofline'];print('$name', d['ms_per_step'], r['kernel'], r['kernels'][r['kernel']]['avg_ms'])"
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof_c2 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config c2 --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > $GRAFT_REPO_ROOT/$OUT/prof_c2.log 2>&1 || { echo "rocprof failed"; tail $GRAFT_REPO_ROOT/$OUT/prof_c2.log; exit 1; }
cd $GRAFT_REPO_ROOT && python tools/prof_summary.py $OUT/prof_c2 > $OUT/kernel_stats_c2.txt 2>&1; head -8 $OUT/kernel_stats_c2.txt | cut -c1-120
