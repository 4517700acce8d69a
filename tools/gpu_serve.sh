# The resident query service: its parity tests and the latency object (tools/latency.py); FULL=1 adds the
# round-3 confirmation (tools/gpu_r03.sh).
set -o pipefail
T=${1:-r03c}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_serve.py -x -v --timeout 120 --timeout-method thread > gpurun_out/$T/pytest_serve.log 2>&1 || exit $?
timeout -k 10 120 python -u tools/latency.py > gpurun_out/$T/latency.json 2> gpurun_out/$T/latency.err || exit $?
timeout -k 10 120 ./tools/latency_serve > gpurun_out/$T/latency_serve.json 2>&1 || exit $?
if [ -n "$FULL" ]; then bash tools/gpu_r03.sh $T; fi
