# A/B of engine builds on NodeCache count 17..32 (tools/nc32_ab.py), each library run twice, interleaved, under
# rocprofv3 --kernel-trace --stats. Usage (on the GPU box): bash tools/gpu_nc32_ab.sh <tag> <lib> [<lib> ...]
# (a lib "head" = the product library); output under gpurun_out/<tag>/.
set -o pipefail
T=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$T
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for i in 1 2; do
  for L in "$@"; do
    if [ "$L" = head ]; then A=""; else A=$R/opendht_amd/$L; fi
    timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${L%.so}_$i -o run -- python3 $R/tools/nc32_ab.py $A > $O/${L%.so}_$i.log 2>&1 || exit 1
  done
done
echo done > $O/done.txt
