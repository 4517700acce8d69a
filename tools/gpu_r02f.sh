set -o pipefail
O=gpurun_out/r02f
mkdir -p $O
timeout -k 10 900 python -u tools/bench_shapes.py 1000000 12500000 > $O/shapes.log 2>&1 || exit $?
