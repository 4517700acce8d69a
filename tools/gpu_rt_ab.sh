# A/B of RoutingTable timings: the product library against libkadgpu_abl.so (built from another source: RT_ABL=1),
# interleaved twice (tools/rt_time.py), after the GPU parity suite when FULL=1.
set -o pipefail
T=${1:-rtab}
mkdir -p gpurun_out/$T
if [ -n "$FULL" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/$T/pytest_gpu.log 2>&1 || exit $?
fi
for r in 1 2; do
  timeout -k 10 200 python -u tools/rt_time.py > gpurun_out/$T/rt_new_$r.json 2>/dev/null || exit $?
  RT_ABL=1 timeout -k 10 200 python -u tools/rt_time.py > gpurun_out/$T/rt_old_$r.json 2>/dev/null || exit $?
done
