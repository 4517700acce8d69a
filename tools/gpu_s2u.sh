# Per-kernel PMC passes over tools/paths_pmc_r02b.py at HEAD (rotated batches).
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/s2u
mkdir -p $O
timeout -k 10 300 python -u tools/paths_pmc_r02b.py > $O/paths_times.log 2>&1 || exit $?
PMC_DIR=s2u/pmc PMC_PROG=tools/paths_pmc_r02b.py PMC_PASSES="FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES;SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU;GRBM_GUI_ACTIVE GRBM_COUNT" bash tools/pmc.sh || exit $?
