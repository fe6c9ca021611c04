set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_sort.py tests/test_gpu_render.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_sort.log 2>&1; echo pytest=$?
tail -2 gpurun_out/pytest_sort.log
timeout -k 10 200 python tools/sortbench.py 30 > gpurun_out/sortbench.txt 2>&1; echo sb=$?
cat gpurun_out/sortbench.txt
timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-sort-bench > gpurun_out/b100.log 2>&1; echo b=$?
