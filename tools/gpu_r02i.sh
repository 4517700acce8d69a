# round-2 path timings and PMC passes (NodeCache two-pass, general lines, headline kernel, rotated batches)
set -o pipefail
O=gpurun_out/r02i
mkdir -p $O
timeout -k 10 300 python -u tools/paths_pmc_r02.py > $O/paths.log 2>&1 || exit $?
PMC_DIR=r02i/pmc PMC_PROG=tools/paths_pmc_r02.py PMC_PASSES="FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES;SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU;GRBM_GUI_ACTIVE GRBM_COUNT" bash tools/pmc.sh
