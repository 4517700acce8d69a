# The count <= 16 NodeCache tests at HEAD, then tools/ncl_ab.py: the product and the baseline libraries alternately,
# twice each, and the ablation build once. Usage (on the GPU box):
#   bash tools/gpu_ncl_ab.sh <tag> <baseline.so under opendht_amd/> ...
set -o pipefail
T=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_line_sets.py tests/test_status_refresh.py tests/test_nc_mirror.py tests/test_config4.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_nc.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 200 python3 tools/ncl_ab.py > $O/head_$i.json 2> $O/head_$i.err || exit $?
  for B in "$@"; do
    timeout -k 10 200 python3 tools/ncl_ab.py $R/opendht_amd/$B > $O/${B%.so}_$i.json 2> $O/${B%.so}_$i.err || exit $?
  done
done
timeout -k 10 200 python3 tools/ncl_ab.py --abl > $O/abl.json 2> $O/abl.err || exit $?
echo done > $O/done.txt
