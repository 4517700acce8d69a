# A/B of a parked NodeCache count <= 16 variant (opendht_amd/libkadgpu_emit.so: branch-free emission in ncl_answer)
# against the product library: its parity tests, then tools/nc_time.py on both.
# Usage (on the GPU box): bash tools/gpu_r04_emit.sh [tag]; output under gpurun_out/<tag>/.
# (The variant library was built from profiles/r04/parked/emit/nc_emit_variant.patch and removed after the A/B.)
set -o pipefail
T=${1:-r04emit}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
L=opendht_amd
cp $L/libkadgpu.so /tmp/base.so || exit 1
cp $L/libkadgpu_emit.so $L/libkadgpu.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_line_sets.py tests/test_nodecache_merge.py tests/test_config4.py tests/test_nc_mirror.py -m gpu > $O/pytest.log 2>&1 || exit $?
timeout -k 10 200 python3 tools/nc_time.py > $O/new.txt 2>&1 || exit $?
cp /tmp/base.so $L/libkadgpu.so
timeout -k 10 200 python3 tools/nc_time.py > $O/base.txt 2>&1 || exit $?
cp $L/libkadgpu_emit.so $L/libkadgpu.so
timeout -k 10 200 python3 tools/nc_time.py > $O/new2.txt 2>&1 || exit $?
cp /tmp/base.so $L/libkadgpu.so
echo done > $O/done.txt
