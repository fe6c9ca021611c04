#!/bin/bash
# One parameterised GPU driver: tools/gpu_run.sh <what> [pytest -k expr | bench args]
#   tests [K]   -m gpu tests (optionally -k K), log in gpurun_out/tests.log
#   all         the round-end driver sequence: every GPU test, smoke(), the default bench line
#   bench ARGS  python bench.py ARGS > gpurun_out/bench.json
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out
mkdir -p $O
what=$1; shift
case "$what" in
tests)
  K=()
  [ -n "$1" ] && K=(-k "$1")
  timeout -k 10 500 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread "${K[@]}" > $O/tests.log 2>&1
  rc=$?; tail -3 $O/tests.log; grep -E "FAILED|Error" $O/tests.log | head -5; exit $rc ;;
all)
  bash tools/gpu_driver_check.sh ;;
bench)
  timeout -k 10 400 python bench.py "$@" > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
  cat $O/bench.json ;;
*) echo "unknown: $what"; exit 2 ;;
esac
