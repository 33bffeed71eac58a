#!/bin/bash
# A/B of the Swimmer config between the default library and a variant
OUT=gpurun_out/c2ab; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -k "c2 or swimmer or api or parity or rows or fused or c1" -x -q --timeout 120 --timeout-method thread > $OUT/t.log 2>&1 || { echo "TESTS FAILED"; tail -30 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
for i in 1 2; do for v in default variant; do
  if [ $v = variant ]; then export MJRL_AMD_LIB=$GRAFT_REPO_ROOT/mjrl_amd/lib/libmjrl_amd_prev.so; else unset MJRL_AMD_LIB; fi
  timeout -k 10 200 python -u bench.py --config c2 --steps 20 --warmup 3 --no-cpu-baseline --no-e2e > $OUT/b_${v}_$i.json 2> $OUT/b_${v}_$i.err || { echo "bench failed"; tail $OUT/b_${v}_$i.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/b_${v}_$i.json'));print('$v', d['ms_per_step'], d.get('eager_ms_per_step'))"
done; done
