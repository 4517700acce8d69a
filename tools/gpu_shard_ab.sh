# A/B of engine builds on the north-star shard kernel (tools/shard_ab.py), each library twice, interleaved, under
# rocprofv3 --kernel-trace --stats. Usage (on the GPU box): bash tools/gpu_shard_ab.sh <tag> <lib|head> ...
set -o pipefail
T=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$T
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for i in 1 2; do
  for L in "$@"; do
    if [ "$L" = head ]; then A=""; else A=$R/opendht_amd/$L; fi
    timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${L%.so}_$i -o run -- python3 $R/tools/shard_ab.py $A > $O/${L%.so}_$i.log 2>&1 || exit 1
  done
done
echo done > $O/done.txt
