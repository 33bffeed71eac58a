#!/bin/bash
# Round 5: the capture-GC fix on the GPU, then the driver's exact suite command.
OUT=gpurun_out/r05a
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 240 python -u tools/capture_gc_repro.py guarded > $OUT/repro_guarded.txt 2>&1 || { echo "REPRO GUARDED FAILED rc=$?"; tail -30 $OUT/repro_guarded.txt; exit 1; }
tail -n 1 $OUT/repro_guarded.txt
timeout -k 10 1000 python3 -m pytest tests/ -x -q -m gpu -p no:cacheprovider > $OUT/pytest_gpu.txt 2>&1 || { echo "SUITE FAILED rc=$?"; tail -40 $OUT/pytest_gpu.txt; exit 1; }
tail -n 3 $OUT/pytest_gpu.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { echo SMOKE FAILED; tail -20 $OUT/smoke.txt; exit 1; }
tail -n 2 $OUT/smoke.txt
echo R05A_DONE
