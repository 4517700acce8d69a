# A/B of the host-pointer batch: in-tree library vs a previous build placed as libkadgpu_abl.so.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/s3e
mkdir -p $O
timeout -k 10 300 python -u tools/host_abi_time.py > $O/new.log 2>&1 || exit $?
RT_ABL=1 timeout -k 10 300 python -u tools/host_abi_time.py > $O/old.log 2>&1 || exit $?
