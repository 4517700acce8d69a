# PMC traffic of the headline kernel on the recipe shard (rotated batches): FETCH_SIZE, WRITE_SIZE, L2 hit passes.
set -o pipefail
R=$(pwd)
PMC_DIR=s2m/pmc BENCH_ARGS="--steps 5 --warmup 2 --no-cpu --no-extras" PMC_PASSES="FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum" bash tools/pmc.sh || exit $?
