set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python tools/timeline.py c3 0 gpurun_out/trace_c3.npz > gpurun_out/timeline_c3.txt 2>&1 && echo TL_OK &&
timeout -k 10 200 python tools/diag.py c3 20 ref,clean > gpurun_out/diag_c3.txt 2>&1 && echo DIAG_OK
