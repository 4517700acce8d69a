# round 2, first measurement session: rotating-batch gather ceiling, the new bench line (rotated
# batches, cold pass, refresh, allgather, CPU baselines), rocprof stats and PMC traffic of the
# rotated headline run. Usage (from the repo root on the GPU box): bash tools/gpu_r02a.sh
set -o pipefail
O=gpurun_out/r02a
mkdir -p $O
timeout -k 10 300 python -u tools/mb_gather.py > $O/mb_gather.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench_k20.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 100 --warmup 10 --no-cpu --no-allgather > $O/bench_k100.log 2>&1 || exit $?
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu --no-extras > $R/$O/prof.log 2>&1 || exit $?
cd $R
PMC_DIR=r02a/pmc BENCH_ARGS="--steps 20 --warmup 5 --no-cpu --no-extras" PMC_PASSES="FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum" bash tools/pmc.sh
