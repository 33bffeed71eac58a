#!/bin/bash
# GPU box: the 1M update with hipGraph replay on vs the default (eager at 1M), alternating
OUT=gpurun_out/${1:-graph1m}; mkdir -p $OUT; export TMPDIR=/tmp
for i in 1 2; do for g in auto on; do
  timeout -k 10 300 python -u bench.py --graph $g --steps 10 --warmup 3 --no-cpu-baseline --no-e2e --no-f32 > $OUT/b_${g}_$i.json 2> $OUT/b_${g}_$i.err || { echo "bench failed"; tail $OUT/b_${g}_$i.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/b_${g}_$i.json'));print('$g', d['ms_per_step'], d.get('hipgraph'), d['roofline']['kernels'][d['roofline']['kernel']]['avg_ms'])"
done; done
