#!/bin/bash
# LLVM scheduling strategies (max-ilp, max-memory-clause) against the default: render tests on
# each, then a same-box frame A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
for v in sILP sMC; do
  bash tools/job_variant_tests.sh $v "tests/test_gpu_render.py" || exit 1
done
bash tools/ab_variants.sh sch0 sILP sMC
