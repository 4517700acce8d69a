set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r02s
mkdir -p $O
timeout -k 10 400 python -u bench.py > $O/bench_default.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu > $O/bench_stats.log 2>&1 || exit $?

