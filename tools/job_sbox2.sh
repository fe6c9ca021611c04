#!/bin/bash
# GS_DRAW_SBOX with the placing pass's box gathers batched: prefix / render tests, then a
# same-box A/B at C3 (twice) and the camera sweep
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
bash tools/job_variant_tests.sh sb1 "tests/test_gpu_prefix.py tests/test_gpu_render.py tests/test_gpu_frames.py tests/test_sh.py" || exit 1
bash tools/ab_variants.sh sb0 sb1 || exit 1
SWEEP=1 bash tools/ab_variants.sh sb0 sb1
