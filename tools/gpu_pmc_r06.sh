# Round-6 per-kernel PMC at HEAD (round 5's script on tools/paths_pmc_r06.py): for every mode of tools/paths_pmc_r06.py, its timings, a
# kernel-trace --stats run (durations per kernel), then one rocprofv3 --pmc run per counter group (kernel-trace only
# besides --pmc). Summarise with tools/pmc_summary.py. Usage (on the GPU box): bash tools/gpu_pmc_r05.sh [tag] [modes]
set -o pipefail
T=${1:-pmc_r06}
MODES=${2:-"shard swarm route"}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$T
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
PASSES="FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES;SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE GRBM_COUNT"
for m in $MODES; do
  timeout -k 10 200 python3 -u $R/tools/paths_pmc_r06.py $m > $O/times_$m.log 2>&1 || exit $?
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_$m -o run -- python3 $R/tools/paths_pmc_r06.py $m > $O/stats_$m.log 2>&1 || exit $?
  IFS=';' read -ra PS <<< "$PASSES"
  i=0
  for line in "${PS[@]}"; do
    i=$((i+1))
    echo "$m pass $i: $line" >> $O/passes.txt
    timeout -s KILL 150 rocprofv3 --pmc $line --kernel-trace --output-format csv -d $O/pmc_$m/p$i -o run -- python3 $R/tools/paths_pmc_r06.py $m > $O/pmc_${m}_p$i.log 2>&1
    rc=$?
    echo "$m pass $i rc=$rc" >> $O/passes.txt
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
echo done > $O/done.txt
