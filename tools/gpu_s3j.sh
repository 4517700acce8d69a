# Confirmation at HEAD: smoke, whole GPU suite, default bench, rocprof kernel stats.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/s3j
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py > $O/bench_default.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --no-cpu --no-extras > $O/prof.log 2>&1 || exit $?
