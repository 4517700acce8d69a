# O(items + slots) radix builder: whole GPU suite + the mirror cost breakdown.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/s2s
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit $?
KAD_DEBUG=1 timeout -k 10 400 python -u tools/bench_mirror.py > $O/mirror.log 2>&1 || exit $?
