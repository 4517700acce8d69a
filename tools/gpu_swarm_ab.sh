# A/B of engine builds on config 5 (tools/bench_swarm.py), each library twice, interleaved; then the swarm tests at
# HEAD. Usage (on the GPU box): bash tools/gpu_swarm_ab.sh <tag> <lib.so under opendht_amd/> ...  ("head": the product)
set -o pipefail
T=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_swarm.py -m gpu -x -q --timeout 280 --timeout-method thread > $O/pytest_swarm.log 2>&1 || exit $?
for i in 1 2; do
  for L in "$@"; do
    if [ "$L" = head ]; then A=""; else A=$R/opendht_amd/$L; fi
    KADGPU_LIB=$A timeout -k 10 200 python3 tools/bench_swarm.py > $O/${L%.so}_$i.json 2> $O/${L%.so}_$i.err || exit $?
  done
done
echo done > $O/done.txt
