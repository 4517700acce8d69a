# Path timings, then PMC passes over tools/paths_pmc.py (one rocprofv3 run per counter group)
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python -u tools/bench_paths.py > $O/paths.log 2>&1 || exit $?
PMC_DIR=pmc_paths PMC_PROG=tools/paths_pmc.py PMC_PASSES="FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES;SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU;GRBM_GUI_ACTIVE GRBM_COUNT" bash tools/pmc.sh
