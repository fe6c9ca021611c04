#!/bin/bash
# Round-2 collection at the final build (GPU box, from the repo root):
#   GPU tests; rocprofv3 trace + FETCH/WRITE/SQ passes + the bench line (collect_profiles.sh);
#   driver-style short runs (20 steps, 5 warm-up) beside the default 100-step one; the other
#   configs and the C5 views; two ranks sharing the GPU, self-spawned and under torchrun.
#   tools/gpu_round2_final.sh a  (tests, profiles, short runs) | b  (configs, views, 2 ranks)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
STAGE=${1:-a}
if [ "$STAGE" = a ]; then
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputests.log 2>&1 || { echo TESTS_FAIL; tail -5 $O/gputests.log; exit 1; }
tail -1 $O/gputests.log
bash tools/collect_profiles.sh r02 > $O/collect.log 2>&1 || { echo COLLECT_FAIL; tail -5 $O/collect.log; exit 1; }
echo COLLECT_OK
for i in 1 2; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-sort-bench > $O/driver_style_$i.json 2>> $O/ds.err || exit 1
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-sort-bench > $O/default_$i.json 2>> $O/ds.err || exit 1
done
python3 -c "
import json
for n in ('driver_style_1', 'default_1', 'driver_style_2', 'default_2'):
    d = json.load(open('$O/%s.json' % n)); print(n, d['steps'], 'steps', d['value'], 'fps')" | tee $O/driver_style_summary.txt
exit 0
fi
bash tools/configs_run.sh > $O/configs_summary.txt 2>&1 || { echo CONFIGS_FAIL; exit 1; }
echo CONFIGS_OK
timeout -k 10 300 python bench.py --gpus 2 --steps 20 --warmup 5 --no-sort-bench > $O/b2.json 2> $O/b2.err || { echo B2_FAIL; exit 1; }
echo B2_OK
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 20 --warmup 5 --no-sort-bench > $O/b2_torchrun.json 2> $O/b2_torchrun.err || { echo B2T_FAIL; tail -5 $O/b2_torchrun.err; exit 1; }
echo B2T_OK
