#!/bin/bash
# One GPU-box session: smoke, GPU parity tests, bench, rocprofv3 kernel-trace of the bench,
# optional A/B timing of kernel variants. Each GPU step runs under its own time limit; a
# crash/timeout (exit >= 124 or a signal) stops the script; plain test failures (pytest exit 1)
# do not stop the bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
step() {  # name, limit, cmd...
  local name=$1 lim=$2; shift 2
  echo "== $name" >> $O/steps.log
  timeout -k 10 $lim "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc" >> $O/steps.log
  if [ $rc -ge 124 ] || [ $rc -gt 128 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
    echo "stopping after $name (rc=$rc)" >> $O/steps.log; exit $rc
  fi
  return 0
}
if [ -z "$NO_TESTS" ]; then
  step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
  step pytest_gpu ${PYTEST_LIMIT:-900} python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-}
fi
step bench 400 python -u bench.py --steps 20 --warmup 5 ${BENCH_EXTRA:-}
if [ -n "$AB" ]; then
  step ab 400 python -u tools/ab_bench.py --variants $AB --rounds 5 --reps 10 ${AB_EXTRA:-}
fi
if [ -z "$NO_PROF" ]; then
  cd /tmp && export TMPDIR=/tmp
  step prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu
fi
if [ -n "$WITH_PMC" ]; then
  bash $R/tools/pmc.sh
fi
echo done >> $O/steps.log
