#!/bin/bash
# GPU box: rocprof of the sharded 125k update and Swimmer, default library vs a variant ($1)
OUT=gpurun_out/${2:-xrp_ab}; mkdir -p $OUT; export TMPDIR=/tmp
for v in default variant; do
  if [ $v = variant ]; then export MJRL_AMD_LIB=$1; else unset MJRL_AMD_LIB; fi
  for c in "p125s:--paths 125 --sharded-path" "c2:--config c2"; do
    name=${c%%:*}; args=${c#*:}
    ( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof_${v}_$name -o run -- python3 $GRAFT_REPO_ROOT/bench.py $args --steps 10 --warmup 3 --no-cpu-baseline --no-e2e --no-f32 > $GRAFT_REPO_ROOT/$OUT/prof_${v}_$name.log 2>&1 ) || { echo "prof failed"; tail $OUT/prof_${v}_$name.log; exit 1; }
    python tools/prof_summary.py $OUT/prof_${v}_$name > $OUT/ks_${v}_$name.txt
    echo "$v $name: $(grep -E 'k_cgm_xrp_f' $OUT/ks_${v}_$name.txt | cut -c75-120)"
  done
done
