#!/bin/bash
# prefix-sort passes 1-3 tile size: GPU prefix/sort tests on the sub8 / sub4 variants, then a
# same-box frame A/B of sub16 (= default) / sub8 / sub4
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
for v in sub8 sub4; do
  bash tools/job_variant_tests.sh $v "tests/test_gpu_prefix.py tests/test_gpu_sort.py" || exit 1
done
bash tools/ab_variants.sh sub16 sub8 sub4
