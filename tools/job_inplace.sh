#!/bin/bash
# in-place blend of wide dense steps (GS_DRAW_INPLACE): render tests on two thresholds, then
# same-box frame A/Bs at C3 and C5 view 7
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
for v in ip128 ip64; do
  bash tools/job_variant_tests.sh $v "tests/test_gpu_render.py tests/test_gpu_frames.py" || exit 1
done
bash tools/ab_variants.sh ip0 ip192 ip128 ip64 || exit 1
BENCH_ARGS="--view 7" bash tools/ab_variants.sh ip0 ip128 ip64
