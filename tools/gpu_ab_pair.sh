set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_render.py tests/test_gpu_frames.py tests/test_sh.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_pair.log 2>&1; echo pytest=$?
tail -2 gpurun_out/pytest_pair.log
bash tools/ab_variants.sh base pair5 pair6
