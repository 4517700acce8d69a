# Per-kernel PMC passes at HEAD over the path workload (tools/paths_pmc.py): its timings, then one rocprofv3 --pmc
# run per counter group (tools/pmc.sh). Summarise with tools/pmc_summary.py (see tools/README.md).
set -o pipefail
T=${1:-pmc_paths}
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/$T
cd $R
timeout -k 10 200 python -u tools/paths_pmc.py > gpurun_out/$T/times.log 2>&1 || exit $?
PMC_DIR=$T/pmc PMC_PROG=tools/paths_pmc.py bash tools/pmc.sh || exit $?
