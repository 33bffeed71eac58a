#!/bin/bash
# Round 5: 1-D slots through the native gather (mjrl_host_gather): staging probe,
# the staged-batch GPU test, and the bench's end-to-end line (no CPU baseline).
OUT=gpurun_out/r05m
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/stage_convert_probe.py 16 none > $OUT/stage_probe.txt 2>&1 || { echo "PROBE FAILED"; tail $OUT/stage_probe.txt; exit 1; }
grep -v amdgpu.ids $OUT/stage_probe.txt
timeout -k 10 300 python3 -m pytest tests/test_gpu_api.py -x -q -p no:cacheprovider -k "staged or from_paths or train_from" > $OUT/pytest.txt 2>&1 || { echo "TESTS FAILED"; tail -30 $OUT/pytest.txt; exit 1; }
tail -n 1 $OUT/pytest.txt
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-f32 > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail $OUT/bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));e=d['e2e_from_host'];t=e['timeline'];print('bench', d['ms_per_step'], 'e2e', e['ms_per_step'], 'staging', e['staging_ms'], 'conv', t['convert_ms'], 'h2d', t['h2d_ms'], t['h2d_busy_ms'], 'upd', t['update_ms'])"
echo R05M_DONE
