#!/bin/bash
# same-box A/B of lib/variants (args), no tests (timing experiments whose output is not checked)
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/ab_variants.sh "$@"
