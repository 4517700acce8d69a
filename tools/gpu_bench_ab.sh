# Headline A/B: bench.py --no-extras --no-cpu --no-allgather with KAD_RT_KERNEL unset and = $AB_VARIANT, interleaved.
set -o pipefail
T=${1:-benchab}
mkdir -p gpurun_out/$T
for r in 1 2 3; do
  timeout -k 10 200 python -u bench.py --no-extras --no-cpu --no-allgather > gpurun_out/$T/default_$r.json 2>/dev/null || exit $?
  KAD_RT_KERNEL=$AB_VARIANT timeout -k 10 200 python -u bench.py --no-extras --no-cpu --no-allgather > gpurun_out/$T/variant_$r.json 2>/dev/null || exit $?
done
