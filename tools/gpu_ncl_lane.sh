# The count <= 16 NodeCache tests, then tools/ncl_lane_ab.py (product forms, then the tools build) and tools/ncl_ab.py
# on the product and the baseline library. Usage (on the GPU box): bash tools/gpu_ncl_lane.sh <tag> [baseline.so]
set -o pipefail
T=$1; B=${2:-libkadgpu_prev.so}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_line_sets.py tests/test_status_refresh.py tests/test_nc_mirror.py tests/test_config4.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_nc.log 2>&1 || exit $?
timeout -k 10 200 python3 tools/ncl_lane_ab.py > $O/lane.json 2> $O/lane.err || exit $?
timeout -k 10 200 python3 tools/ncl_lane_ab.py --abl > $O/lane_abl.json 2> $O/lane_abl.err || exit $?
for i in 1 2; do
  timeout -k 10 200 python3 tools/ncl_ab.py > $O/head_$i.json 2> $O/head_$i.err || exit $?
  timeout -k 10 200 python3 tools/ncl_ab.py $R/opendht_amd/$B > $O/${B%.so}_$i.json 2> $O/${B%.so}_$i.err || exit $?
done
echo done > $O/done.txt
