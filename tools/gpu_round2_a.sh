set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && echo PYTEST_OK &&
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/b20.log 2>gpurun_out/b20.err && echo B20_OK &&
timeout -k 10 200 python bench.py --gpus 1 --steps 100 --warmup 10 --no-cpu-baseline --no-sort-bench > gpurun_out/b100.log 2>&1 && echo B100_OK &&
timeout -k 10 300 python bench.py --gpus 2 --steps 20 --warmup 5 --no-sort-bench > gpurun_out/b2.log 2>&1 && echo B2_OK
