#!/bin/bash
# GPU box: the whole GPU suite on the release build, then the smoke.
OUT=gpurun_out/${1:-suite}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/t.log 2>&1 \
  || { echo "SUITE FAILED"; grep -E "FAILED|Error|error" $OUT/t.log | head -30; tail -5 $OUT/t.log; exit 1; }
tail -n 2 $OUT/t.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 $OUT/smoke.log; exit 1; }
tail -n 1 $OUT/smoke.log
echo SUITE_DONE
