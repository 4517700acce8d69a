# One A/B session of RoutingTable kernel variants (tools/ab_kernels.py): AB_COUNTS, AB_VARIANTS.
set -o pipefail
T=${1:-ab}
mkdir -p gpurun_out/$T
timeout -k 10 400 python -u tools/ab_kernels.py ${AB_COUNTS:-17,24,32} ${AB_VARIANTS:-,wl32lane} > gpurun_out/$T/ab.json 2> gpurun_out/$T/ab.err || exit $?
