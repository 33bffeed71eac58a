#!/bin/bash
# GPU box: Swimmer bench (k_fused FVP average) over library variants, alternating:
#   bash tools/gpu_var.sh OUT base:mjrl_amd/lib/libmjrl_amd_base.so pa:mjrl_amd/lib/libmjrl_amd_pa.so ...
# ("default" = the in-tree library)
OUT=gpurun_out/${1:-var}; shift
mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2; do for spec in default "$@"; do
  name=${spec%%:*}; lib=${spec#*:}
  if [ $name = default ]; then unset MJRL_AMD_LIB; else export MJRL_AMD_LIB=$lib; fi
  timeout -k 10 200 python -u bench.py --config c2 --steps 20 --warmup 3 --no-cpu-baseline --no-e2e > $OUT/b_${name}_$i.json 2> $OUT/b_${name}_$i.err || { echo "bench $name failed"; tail $OUT/b_${name}_$i.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/b_${name}_$i.json'));r=d['roofline'];print('%-8s'%'$name', d['ms_per_step'], r['kernel'], r['kernels'][r['kernel']]['avg_ms'])"
done; done
