#!/bin/bash
# GPU box: mjrl_gae against its timing-ablation builds, built beforehand with
#   python -m mjrl_amd.build --tag _nofwd --extra=-DMJRL_GAE_ABL_NOFWD   (and _noload / _nochain)
# Usage: bash tools/gpu_gae_abl.sh <tag>
OUT=gpurun_out/${1:-gae_abl}
mkdir -p $OUT
export GAE_PROBE_ONLY=1
for v in "" _nofwd _noload _nochain; do
  if [ -z "$v" ]; then LIBV=mjrl_amd/lib/libmjrl_amd.so; NC=0; else LIBV=mjrl_amd/lib/libmjrl_amd$v.so; NC=1; fi
  echo "build: ${v:-default}"
  MJRL_AMD_LIB=$LIBV MJRL_AMD_ALLOW_ABLATION=1 GAE_PROBE_NOCHECK=$NC timeout -k 10 120 python3 -u tools/gae_probe.py > $OUT/gae${v:-_default}.txt 2>&1 || { echo "probe $v failed"; tail $OUT/gae${v:-_default}.txt; exit 1; }
  grep -v amdgpu.ids $OUT/gae${v:-_default}.txt | cut -c1-45
done
