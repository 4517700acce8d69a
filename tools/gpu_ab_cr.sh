set -o pipefail
mkdir -p gpurun_out/ab_cr
timeout -k 10 200 python -u tools/ab_bench.py --variants default,ws_cr --rounds 9 --reps 20 > gpurun_out/ab_cr/ab_bench.json 2> gpurun_out/ab_cr/ab_bench.err || exit $?
AB_VARIANT=ws_cr bash tools/gpu_bench_ab.sh ab_cr
