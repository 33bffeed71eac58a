#!/bin/bash
# GPU box: split / parity tests on the default library, then the default bench
# (1M rows) alternating the libraries given as arguments (paths relative to the
# repo; "default" = the in-tree default), with rocprofv3 kernel stats of each.
OUT=gpurun_out/ab3
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $OUT/t.log 2>&1 || { echo "TESTS FAILED"; tail -20 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
for i in 1 2; do
  for v in "$@"; do
    if [ $v = default ]; then unset MJRL_AMD_LIB; else export MJRL_AMD_LIB=$GRAFT_REPO_ROOT/$v; fi
    tag=$(basename $v .so)
    timeout -k 10 200 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-e2e --no-f32 > $OUT/b_${tag}_$i.json 2> $OUT/b_${tag}_$i.err || { echo "bench $v failed"; tail $OUT/b_${tag}_$i.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/b_${tag}_$i.json'));print('$tag', d['ms_per_step'], d['roofline']['kernels']['k_kx<32,12,FVP>']['avg_ms'])"
  done
done
for v in "$@"; do
  if [ $v = default ]; then unset MJRL_AMD_LIB; else export MJRL_AMD_LIB=$GRAFT_REPO_ROOT/$v; fi
  tag=$(basename $v .so)
  ( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/p_$tag -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --no-f32 > $GRAFT_REPO_ROOT/$OUT/p_$tag.log 2>&1 ) || { echo "prof $v failed"; exit 1; }
  echo "== $tag"; python tools/prof_summary.py $OUT/p_$tag | sed -n 2,5p | cut -c1-50,70-
done
