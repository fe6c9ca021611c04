#!/bin/bash
# cull boxes in sorted order for prefix-sorted frames (GS_DRAW_SBOX): prefix / render / frame
# tests, then same-box A/Bs at C3 and C5 view 7
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
bash tools/job_variant_tests.sh sb1 "tests/test_gpu_prefix.py tests/test_gpu_render.py tests/test_gpu_frames.py tests/test_sh.py" || exit 1
bash tools/ab_variants.sh sb0 sb1 || exit 1
BENCH_ARGS="--view 7" bash tools/ab_variants.sh sb0 sb1
