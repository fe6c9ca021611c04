#!/bin/bash
# the round's last build: every config / mode / C5 view bench line, then four ranks sharing the
# one leased GPU (self-spawned and under torch.distributed.run)
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/configs_run.sh > gpurun_out/configs_summary.txt 2>&1 || { echo CONFIGS_FAIL; tail -5 gpurun_out/configs_summary.txt; exit 1; }
cat gpurun_out/configs_summary.txt
bash tools/gpu_ranks4.sh || exit 1
tail -1 gpurun_out/b4_spawn.log; tail -1 gpurun_out/b4_torchrun.log
