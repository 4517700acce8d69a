#!/bin/bash
# One GPU-box session: smoke, GPU parity tests, bench, rocprofv3 kernel-trace of the bench.
# Each GPU step runs under its own time limit; a crash/timeout (exit >= 124 or a signal)
# stops the script; plain test failures (pytest exit 1) do not stop the bench.
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
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu ${PYTEST_LIMIT:-900} python -m pytest tests -m gpu -q ${PYTEST_ARGS:-}
step bench 400 python bench.py --steps 20 --warmup 5
if [ -z "$NO_PROF" ]; then
  cd /tmp && export TMPDIR=/tmp
  step prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu
fi

if [ -n "$WITH_PMC" ]; then
  bash $R/tools/pmc.sh
fi
echo done >> $O/steps.log
