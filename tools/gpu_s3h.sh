# rocprof kernel stats of the headline alone (bench.py --no-extras --no-cpu: warmup + timed steps, every rt_ws_kernel
# launch a 1M-query step on the bench shard), beside the live HIP-event average it prints.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/s3h
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --no-cpu --no-extras > $O/prof.log 2>&1 || exit $?
