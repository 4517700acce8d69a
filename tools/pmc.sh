#!/bin/bash
# PMC passes over a short bench run (one rocprofv3 invocation per counter group, kernel-trace
# only besides --pmc, as the MI355X guide prescribes). Output: gpurun_out/pmc/<pass>/...
# PMC_PASSES="A B;C D" overrides the pass list (';' between passes); PMC_PROG="tools/x.py args"
# profiles another script instead of bench.py.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${PMC_DIR:-pmc}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
ARGS=${BENCH_ARGS:---steps 5 --warmup 2 --no-cpu}
DEFAULT="FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES;SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD;GRBM_GUI_ACTIVE GRBM_COUNT;TA_BUSY_avr TA_TA_BUSY_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"
IFS=';' read -ra PASSES <<< "${PMC_PASSES:-$DEFAULT}"
i=0
for line in "${PASSES[@]}"; do
  [ -z "$line" ] && continue
  i=$((i+1))
  echo "pass $i: $line" >> $O/passes.txt
  timeout -s KILL 120 rocprofv3 --pmc $line --kernel-trace --output-format csv -d $O/p$i -o run -- python3 ${PMC_PROG:+$R/}${PMC_PROG:-$R/bench.py $ARGS} > $O/p$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc" >> $O/passes.txt
  if [ $rc -ne 0 ]; then exit $rc; fi
done
echo done >> $O/passes.txt
