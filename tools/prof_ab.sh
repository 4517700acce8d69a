#!/bin/bash
# GPU parity tests, then an A/B timing of RoutingTable kernel variants under rocprofv3 kernel-trace.
# usage (on the box): VARIANTS=rec,lane bash tools/prof_ab.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > $O/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> $O/steps.log
  if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then exit $rc; fi
fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/tools/ab_bench.py --variants ${VARIANTS:-rec,lane} --rounds 3 --reps 5 ${AB_EXTRA:-} > $O/ab.log 2>&1
echo "ab rc=$?" >> $O/steps.log
python3 - <<'PY' >> $O/ab.log
import csv, os
p = os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "gpurun_out/prof/run_kernel_stats.csv")
for r in csv.DictReader(open(p)):
    print("KSTAT", r["Name"].split("(")[0][-60:], r["Name"].split("<")[1].split(">")[0] if "<" in r["Name"] else "", r["Calls"], r["AverageNs"], r["MinNs"], r["MaxNs"])
PY
