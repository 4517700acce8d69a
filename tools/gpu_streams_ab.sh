# A/B of the row-store policy: the product library (non-temporal rows) against libkadgpu_abl.so built with
# ABL_DEFS=-DKAD_PLAIN_STREAMS, RoutingTable (rt_time.py) and NodeCache (nc_time.py) timings, interleaved twice.
set -o pipefail
T=${1:-streamsab}
mkdir -p gpurun_out/$T
for r in 1 2; do
  timeout -k 10 200 python -u tools/rt_time.py > gpurun_out/$T/rt_nt_$r.json 2>/dev/null || exit $?
  RT_ABL=1 timeout -k 10 200 python -u tools/rt_time.py > gpurun_out/$T/rt_plain_$r.json 2>/dev/null || exit $?
  timeout -k 10 300 python -u tools/nc_time.py > gpurun_out/$T/nc_nt_$r.json 2>/dev/null || exit $?
  NC_ABL=1 timeout -k 10 300 python -u tools/nc_time.py > gpurun_out/$T/nc_plain_$r.json 2>/dev/null || exit $?
done
