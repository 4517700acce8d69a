# Round-4 A/B of two kernel variants kept out of the source until their GPU parity holds: the NodeCache count
# 17..32 line kernel with DPP / ds_swizzle octet moves (opendht_amd/libkadgpu_nc.so) and the small refresh with
# per-bucket offsets for up to 128 host buckets (libkadgpu_rf.so, libkadgpu_rf_abl.so). Each variant's parity tests
# run against it, then the timing tools against it and against the product library.
# Usage (on the GPU box): bash tools/gpu_r04_parked.sh [tag]; output under gpurun_out/<tag>/.
# (The variant libraries were built from the patches under profiles/r04/parked/ and removed after the A/B.)
set -o pipefail
T=${1:-r04parked}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
L=opendht_amd
cp $L/libkadgpu.so /tmp/base.so && cp $L/libkadgpu_abl.so /tmp/base_abl.so || exit 1
timeout -k 10 60 ./tools/oct_check > $O/oct.txt 2>&1 || exit $?
# NodeCache 17..32
cp $L/libkadgpu_nc.so $L/libkadgpu.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_nc_lines32.py tests/test_nodecache_merge.py tests/test_config4.py -m gpu > $O/nc_pytest.log 2>&1 || exit $?
timeout -k 10 200 python3 tools/nc_time.py > $O/nc_new.txt 2>&1 || exit $?
cp /tmp/base.so $L/libkadgpu.so
timeout -k 10 200 python3 tools/nc_time.py > $O/nc_base.txt 2>&1 || exit $?
# small refresh
cp $L/libkadgpu_rf.so $L/libkadgpu.so && cp $L/libkadgpu_rf_abl.so $L/libkadgpu_abl.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_status_refresh.py tests/test_line_sets.py -m gpu > $O/rf_pytest.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/rf_new -o t -- python3 $R/tools/rf_trace.py > $O/rf_new.log 2>&1 || exit $?
cp /tmp/base_abl.so $R/$L/libkadgpu_abl.so && cp /tmp/base.so $R/$L/libkadgpu.so
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/rf_base -o t -- python3 $R/tools/rf_trace.py > $O/rf_base.log 2>&1 || exit $?
echo done > $O/done.txt
