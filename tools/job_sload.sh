#!/bin/bash
# survivor broadcast by scalar loads (GS_DRAW_SLOAD): render + frame tests, then same-box A/Bs at
# C3 and C5 view 7
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
bash tools/job_variant_tests.sh sl1 "tests/test_gpu_render.py tests/test_gpu_frames.py tests/test_gpu_prefix.py" || exit 1
bash tools/ab_variants.sh sl0 sl1 || exit 1
BENCH_ARGS="--view 7" bash tools/ab_variants.sh sl0 sl1
