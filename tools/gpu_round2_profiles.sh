set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/collect_profiles.sh r02 > gpurun_out/collect.log 2>&1 || { echo COLLECT_FAIL; tail -5 gpurun_out/collect.log; exit 1; }
echo COLLECT_OK
bash tools/configs_run.sh > gpurun_out/configs_summary.txt 2>&1 || { echo CONFIGS_FAIL; exit 1; }
echo CONFIGS_OK
timeout -k 10 300 python bench.py --gpus 2 --steps 20 --warmup 5 --no-sort-bench > gpurun_out/b2.log 2>&1 && echo B2_OK
