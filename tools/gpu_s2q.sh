# Mirror cost breakdown (KAD_DEBUG phase times) on the bench shard.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/s2q
mkdir -p $O
KAD_DEBUG=1 timeout -k 10 400 python -u tools/bench_mirror.py > $O/mirror.log 2>&1 || exit $?
