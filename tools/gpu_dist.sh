#!/bin/bash
# GPU box: sharded-update tests (2 ranks on the one GPU over gloo) and a 2-rank
# rehearsal of bench.py's N > 1 path (gloo; the driver's multi-GPU runs use RCCL)
OUT=gpurun_out/${1:-dist}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py -x -v --timeout 200 --timeout-method thread > $OUT/dist.log 2>&1; rc=$?; echo "dist rc=$rc"; grep -E "PASS|FAIL|Error" $OUT/dist.log | head; [ $rc -eq 0 ] || exit 1
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 3 --warmup 1 --backend gloo > $OUT/bench2.json 2> $OUT/bench2.err; rc=$?; echo "bench2 rc=$rc"; cat $OUT/bench2.json | head -c 600; echo; [ $rc -eq 0 ] || tail -20 $OUT/bench2.err
