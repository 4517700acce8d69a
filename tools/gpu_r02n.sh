set -o pipefail
R=$(pwd)
PMC_DIR=r02n/calib PMC_PASSES="FETCH_SIZE;WRITE_SIZE" PMC_PROG=tools/mb_calib.py bash tools/pmc.sh || exit $?
cd $R
PMC_DIR=r02n/bench PMC_PASSES="FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum" bash tools/pmc.sh || exit $?
cd $R
for k in "k_lane<4>" "k_lane<8>"; do python3 tools/parse_pmc.py gpurun_out/r02n/calib "$k" > "gpurun_out/r02n/calib_$k.json" || exit $?; done
python3 tools/parse_pmc.py gpurun_out/r02n/bench rt_ws_kernel > gpurun_out/r02n/bench_ws.json || exit $?
cd /tmp && export TMPDIR=/tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r02n/stats -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu > $R/gpurun_out/r02n/bench_stats.log 2>&1 || exit $?
