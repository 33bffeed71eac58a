#!/bin/bash
# GPU box: the whole GPU suite on the release build, then the smoke.
OUT=gpurun_out/${1:-suite}
mkdir -p $OUT
export TMPDIR=/tmp
# the driver's exact command line (no pytest-timeout plugin: it changes the process)
timeout -k 10 1000 python3 -m pytest tests/ -x -q -m gpu -p no:cacheprovider > $OUT/t.log 2>&1 \
  || { echo "SUITE FAILED"; grep -E "FAILED|Error|error" $OUT/t.log | head -30; tail -5 $OUT/t.log; exit 1; }
tail -n 2 $OUT/t.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 $OUT/smoke.log; exit 1; }
tail -n 1 $OUT/smoke.log
echo SUITE_DONE
