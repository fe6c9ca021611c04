set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && echo PYTEST_OK &&
timeout -k 10 200 python bench.py --gpus 1 --steps 100 --warmup 10 --no-cpu-baseline --no-sort-bench > gpurun_out/b100.log 2>&1 && echo B100_OK
