#!/bin/bash
# four ranks sharing the one leased GPU: self-spawned, then under torch.distributed.run (the
# driver's N > 1 launch); each rank renders its own C5 view, the line is the max over ranks
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 300 python bench.py --gpus 4 --steps 20 --warmup 5 --no-sort-bench > $O/b4_spawn.log 2>&1 || { echo SPAWN_FAIL; tail -5 $O/b4_spawn.log; exit 1; }
echo SPAWN_OK
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29517 \
    bench.py --gpus 4 --steps 20 --warmup 5 --no-sort-bench > $O/b4_torchrun.log 2>&1 || { echo TORCHRUN_FAIL; tail -5 $O/b4_torchrun.log; exit 1; }
echo TORCHRUN_OK
