#!/bin/bash
# One parameterised GPU driver: tools/gpu_run.sh <what> [pytest -k expr | bench args]
#   tests [K]   -m gpu tests (optionally -k K), log in gpurun_out/tests.log
#   all         the round-end driver sequence: every GPU test, smoke(), the default bench line
#   bench ARGS  python bench.py ARGS > gpurun_out/bench.json
#   ab K [ARGS] tests -k K on the working tree's library, then bench A (lib/libgsplat_hip_old.so,
#               tools/build_ab.sh) / B (the working tree's) twice each, interleaved
#   variants N.. same-box A/B of lib/variants/N.so (tools/variants.sh)
#   lab V..     experiments: TESTV / TL / SWEEPV (see the mode) and a same-box A/B of lib/variants/V.so
#   configs     bench lines of C4, SH, clean, fast exp, C2 and the eight C5 views
#   profiles T  the round's rocprofv3 collection (trace by pass, FETCH / WRITE / SQ, C2, view 4)
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
ab)
  # same-box A/B: lib/libgsplat_hip_old.so (A: tools/build_ab.sh's HEAD build) against the working
  # tree's lib/libgsplat_hip.so (B); the GPU tests matching $1 run on B first
  L=openglgaussiansplattingrenderer_amd/lib
  cp $L/libgsplat_hip.so /tmp/lib_b.so
  if [ -n "$1" ]; then
    timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread -k "$1" > $O/ab_tests.log 2>&1 || { tail -5 $O/ab_tests.log; exit 1; }
    tail -1 $O/ab_tests.log
  fi
  shift
  one() {
    # (AB_SWEEP=1: with the camera sweeps, their ratios against the same poses static printed too)
    local sw=--no-sweep; [ -n "$AB_SWEEP" ] && sw=
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-sort-bench --no-facade $sw "$@" > $O/ab_$v$i.json 2> $O/ab.err || { tail -5 $O/ab.err; return 1; }
    python3 -c "
import json; d=json.load(open('$O/ab_$v$i.json')); fr=d['frame']
print('$v', d['value'], 'serial', fr['serial_ms_per_frame'], 'draw', d['roofline']['avg_launch_ms'], {k: round(x, 4) for k, x in fr['stage_ms'].items()})
sw = fr.get('camera_sweep') or {}
for k, r in sw.items():
    if isinstance(r, dict) and 'prefix' in r:
        print('   sweep', k, 'vs_static_same_poses', r['prefix']['vs_static_same_poses'], 'again', r['prefix']['rendered_again'], 'kept', r['prefix']['kept_frac_last'], 'fps', r['prefix']['frames_per_s'])"
  }
  for i in 1 2; do
    v=A; cp $L/libgsplat_hip_old.so $L/libgsplat_hip.so; one "$@" || break
    v=B; cp /tmp/lib_b.so $L/libgsplat_hip.so; one "$@" || break
  done
  cp /tmp/lib_b.so $L/libgsplat_hip.so ;;
variants)
  # same-box A/B of lib/variants/NAME.so builds (tools/variants.sh NAME -DFLAG=...), in the given order, twice
  bash tools/ab_variants.sh "$@" ;;
lab)
  # experiment runs: TESTV=NAME every GPU test on lib/variants/NAME.so; TL="a b" light-trace
  # timelines (tools/timeline.py, GS_FLAG_DRAW_TRACE) of those variants; then a same-box A/B of the
  # variants given as arguments (tools/ab_variants.sh) and SWEEPV="a b" another with the camera sweeps
  L=openglgaussiansplattingrenderer_amd/lib
  cp $L/libgsplat_hip.so /tmp/orig.so
  if [ -n "$TESTV" ]; then
    cp $L/variants/$TESTV.so $L/libgsplat_hip.so
    timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > $O/tests_$TESTV.log 2>&1
    rc=$?; tail -2 $O/tests_$TESTV.log
    cp /tmp/orig.so $L/libgsplat_hip.so
    [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/tests_$TESTV.log | head -5; exit 1; }
  fi
  for v in $TL; do
    cp $L/variants/$v.so $L/libgsplat_hip.so
    GS_LIGHT_TRACE=1 timeout -k 10 200 python tools/timeline.py c3 > $O/timeline_$v.txt 2>&1 || { cp /tmp/orig.so $L/libgsplat_hip.so; exit 1; }
    sed -n 3,6p $O/timeline_$v.txt
  done
  cp /tmp/orig.so $L/libgsplat_hip.so
  [ $# -gt 0 ] && { bash tools/ab_variants.sh "$@" || exit 1; }
  [ -n "$SWEEPV" ] && SWEEP=1 bash tools/ab_variants.sh $SWEEPV
  exit 0 ;;
configs)
  # bench lines of the other configs / modes and every C5 view (pose k), one GPU -> gpurun_out/configs/
  C=$O/configs; mkdir -p $C
  b() { timeout -k 10 200 python bench.py --no-cpu-baseline --no-sort-bench --no-sweep $1 > $C/$2.json 2>> $C/err.log || return 1
    python3 -c "
import json; d=json.load(open('$C/$2.json')); fr=d['frame']
print('$2', d['value'], 'fps', d['ms_per_step'], 'ms; serial', fr['serial_ms_per_frame'], 'E', fr['E'], fr['stage_ms'], 'draw frac', d['roofline']['frac'])"; }
  b "--config c4" c4 && b "--sh" sh && b "--clean" clean && b "--fast-exp" fastexp && b "--config c2" c2 || exit 1
  for k in 0 1 2 3 4 5 6 7; do b "--view $k" view$k || exit 1; done ;;
profiles)
  # the round's profile collection (TAG, e.g. r04): GPU tests, the kernel trace of the default bench
  # command split by pass, FETCH / WRITE / SQ passes (separate runs), C2 and C5 view 4 traced, the SH
  # line and the bench line after -> gpurun_out/prof_TAG/ (copy the summaries into profiles/TAG/: bench.py reads the newest
# profiles/rNN/pmc_summary.json and sort_64M_pmc.json)
  TAG=${1:-r05}; R=$(pwd); P=$R/$O/prof_$TAG; mkdir -p $P
  timeout -k 10 500 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests > $O/prof_tests.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/prof_tests.log; exit 1; }
  tail -1 $O/prof_tests.log
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $P/trace -o run --output-format csv -- \
      python3 $R/bench.py --no-cpu-baseline --no-sweep > $P/bench_under_trace.json 2> $P/trace.err || { echo TRACE_FAIL; exit 1; }
  python3 $R/tools/trace_passes.py $P/trace/run_kernel_trace.csv 50 10 100 > $P/bench_trace_by_pass.txt
  python3 $R/tools/trace_summary.py $P/trace/run_kernel_trace.csv > $P/bench_kernel_trace_summary.txt
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $P/fetch -o run --output-format csv -- \
      python3 $R/tools/frames.py c3 0 6 > /dev/null 2> $P/fetch.err || { echo FETCH_FAIL; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $P/write -o run --output-format csv -- \
      python3 $R/tools/frames.py c3 0 6 > /dev/null 2> $P/write.err || { echo WRITE_FAIL; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU \
      SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_SALU -d $P/sq -o run --output-format csv -- \
      python3 $R/tools/frames.py c3 0 6 > /dev/null 2> $P/sq.err || { echo SQ_FAIL; exit 1; }
  python3 $R/tools/pmc_summary.py $P/fetch/run_counter_collection.csv $P/write/run_counter_collection.csv \
      $P/pmc_summary.json $P/sq/run_counter_collection.csv > $P/pmc_summary.txt
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $P/sfetch -o run --output-format csv -- \
      python3 $R/tools/bigsort.py > $P/bigsort_fetch.json 2> $P/sfetch.err || { echo SFETCH_FAIL; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $P/swrite -o run --output-format csv -- \
      python3 $R/tools/bigsort.py > $P/bigsort_write.json 2> $P/swrite.err || { echo SWRITE_FAIL; exit 1; }
  python3 $R/tools/sort_pmc_summary.py $P/sfetch/run_counter_collection.csv $P/swrite/run_counter_collection.csv \
      $P/sort_64M_pmc.json > $P/sort_64M_pmc.txt
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $P/trace_c2 -o run --output-format csv -- \
      python3 $R/bench.py --config c2 --no-cpu-baseline --no-sort-bench > $P/c2_under_trace.json 2> $P/c2.err || { echo C2_FAIL; exit 1; }
  python3 $R/tools/trace_passes.py $P/trace_c2/run_kernel_trace.csv 50 10 100 > $P/c2_trace_by_pass.txt
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $P/trace_v4 -o run --output-format csv -- \
      python3 $R/bench.py --view 4 --no-cpu-baseline --no-sort-bench --no-sweep > $P/v4_under_trace.json 2> $P/v4.err || { echo V4_FAIL; exit 1; }
  python3 $R/tools/trace_passes.py $P/trace_v4/run_kernel_trace.csv 50 10 100 > $P/v4_trace_by_pass.txt
  cd $R
  timeout -k 10 200 python3 bench.py --sh --no-cpu-baseline --no-sort-bench --no-sweep --no-facade > $P/sh.json 2> $P/sh.err || { echo SH_FAIL; exit 1; }
  timeout -k 10 200 python3 tools/valu_account.py c3 > $P/valu_account.txt 2> $P/valu.err || { echo VALU_FAIL; exit 1; }
  timeout -k 10 300 python3 bench.py > $P/bench_latest.json 2> $P/bench.err || { echo BENCH_FAIL; exit 1; }
  echo done ;;
*) echo "unknown: $what"; exit 2 ;;
esac
