#!/bin/bash
# The one GPU-box runner: the named steps in order, each under its own time limit, output under
# gpurun_out/$TAG/.  Stops at the first step that dies by a signal / time limit / abort (rc >= 124: nothing
# more may touch the GPU in that call); goes on after an ordinary failure (rc 1-123, e.g. a failing test)
# and exits with it.
#
#   usage: gpurun -- 'TAG=r06a bash tools/gpu_run.sh STEP [STEP ...]'
#
# steps:
#   tests[=PYTEST_ARGS]  the GPU suite (default: tests -m gpu), or the given files / -k filter
#   smoke                __graft_entry__.smoke()
#   bench[=BENCH_ARGS]   bench.py's JSON line -> bench.json (default: the driver's default run)
#   trace                C2 step kernel trace -> trace/step_summary.txt            (tools/gpu_trace.sh)
#   inftrace             inference kernel traces B=1 / B=16 / 436x1024 -> inf/     (tools/gpu_inftrace.sh)
#   layertable           per-conv-op table of one C2 step -> layertable.jsonl       (tools/layertable.py)
#   ab=ARMS              same-box C2 step A/B of env settings, e.g. ab="default VST_X=0"  (tools/ab_step.sh)
#   infab=ARMS           same-box inference A/B                                      (tools/gpu_infab.sh)
#   pmc[=OPS]            counter passes over the ResnetBlock conv ops + record       (tools/profile_counters.sh)
#   wgradab              same-box kernel A/B of the ResnetBlock weight gradient routes    (tools/wgrad_ab.sh)
#   sgab=ARMS            same-box StarGAN C4 line A/B                                 (tools/sg_ab.sh)
#   fnab=FN:ARMS         same-box A/B of one bench.py line function, e.g. fnab="c3_train_fps:default X=1"  (tools/fn_ab.sh)
#   sgtrace | jstrace | mgtrace | rafttrace | c3trace   secondary-line kernel traces
#   stamp                the kernel-source stamp of the tree being run
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${TAG:-run}
O=gpurun_out/$TAG
mkdir -p $O
final=0
for step in "$@"; do
  name=${step%%=*}
  arg=""
  [ "$name" != "$step" ] && arg=${step#*=}
  echo "=== $step"
  case $name in
    tests)
      timeout -k 10 900 python3 -u -m pytest -q --timeout 280 --timeout-method thread -p no:cacheprovider \
        ${arg:-tests -m gpu} > $O/tests.log 2>&1
      rc=$?; tail -3 $O/tests.log ;;
    smoke)
      timeout -k 10 300 python3 -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1
      rc=$?; tail -2 $O/smoke.log ;;
    bench)
      timeout -k 10 600 python3 bench.py $arg > $O/bench.json 2> $O/bench.err
      rc=$?; tail -c 600 $O/bench.json; [ $rc -ne 0 ] && tail -20 $O/bench.err ;;
    trace)
      TAG=$TAG/trace bash tools/gpu_trace.sh; rc=$? ;;
    inftrace)
      TAG=$TAG/inf bash tools/gpu_inftrace.sh > /dev/null; rc=$? ;;
    layertable)
      timeout -k 10 300 python3 -u tools/layertable.py 3 > $O/layertable.jsonl 2> $O/layertable.err
      rc=$?; tail -1 $O/layertable.jsonl; [ $rc -ne 0 ] && tail -20 $O/layertable.err ;;
    ab)
      ARMS="$arg" TAG=$TAG/ab bash tools/ab_step.sh; rc=$? ;;
    infab)
      ARMS="$arg" TAG=$TAG/infab bash tools/gpu_infab.sh; rc=$? ;;
    pmc)
      TAG=$TAG/pmc OPS="${arg:-fprop dgrad wgrad_nhwc wgrad_pre c0 warp}" bash tools/profile_counters.sh &&
        timeout -k 10 120 python3 tools/pmc_resblock.py $O/pmc $O/pmc/conv 5
      rc=$? ;;
    wgradab) TAG=$TAG/wgab bash tools/wgrad_ab.sh; rc=$? ;;
    sgab) ARMS="$arg" TAG=$TAG/sgab bash tools/sg_ab.sh; rc=$? ;;
    fnab) FN="${arg%%:*}" ARMS="${arg#*:}" TAG=$TAG/fnab_${arg%%:*} bash tools/fn_ab.sh; rc=$? ;;
    sgtrace) TAG=$TAG/sg bash tools/gpu_sgtrace.sh; rc=$? ;;
    jstrace) TAG=$TAG/js bash tools/gpu_jstrace.sh; rc=$? ;;
    mgtrace) TAG=$TAG/mg bash tools/gpu_mgtrace.sh; rc=$? ;;
    rafttrace) TAG=$TAG/raft bash tools/gpu_rafttrace.sh; rc=$? ;;
    c3trace) TAG=$TAG/c3 bash tools/gpu_c3trace.sh; rc=$? ;;
    stamp)
      python3 -c "import sys; sys.path.insert(0, '.'); from gbvst import _lib; print(_lib.source_stamp())" | tee $O/stamp.txt
      rc=$? ;;
    *) echo "unknown step $name"; rc=2 ;;
  esac
  echo "=== rc=$rc"
  if [ $rc -ge 124 ]; then exit $rc; fi
  if [ $rc -ne 0 ]; then final=$rc; fi
done
exit $final
