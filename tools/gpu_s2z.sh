# A/B: rt timings with the in-tree library and with a previous build placed as libkadgpu_abl.so.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/s2z
mkdir -p $O
timeout -k 10 300 python -u tools/rt_time.py > $O/new1.log 2>&1 || exit $?
RT_ABL=1 timeout -k 10 300 python -u tools/rt_time.py > $O/old1.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/rt_time.py > $O/new2.log 2>&1 || exit $?
RT_ABL=1 timeout -k 10 300 python -u tools/rt_time.py > $O/old2.log 2>&1 || exit $?
