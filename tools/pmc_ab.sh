#!/bin/bash
# PMC passes over tools/ab_bench.py for one variant: VARIANT=rec|lane  (output gpurun_out/pmc_<variant>)
R=${GRAFT_REPO_ROOT:-$(pwd)}
V=${VARIANT:-lane}
O=$R/gpurun_out/pmc_$V
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
while read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $line --kernel-trace --output-format csv -d $O/p$i -o run -- python3 $R/tools/ab_bench.py --variants $V --rounds 1 --reps 3 > $O/p$i.log 2>&1
  rc=$?
  echo "pass $i ($line) rc=$rc" >> $O/passes.txt
  if [ $rc -ge 124 ]; then exit $rc; fi
done <<'PASSES'
FETCH_SIZE
TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VMEM_WR
SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM
GRBM_GUI_ACTIVE TA_BUSY_avr TA_TA_BUSY_sum
PASSES
