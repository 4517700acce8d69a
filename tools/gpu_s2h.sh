# NodeCache two-pass breakdown: ablations with the pass-1 marked share, and the per-kernel trace of nc_abl.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/s2h
mkdir -p $O
timeout -k 10 300 python -u tools/nc_abl.py > $O/nc_abl.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/tools/nc_abl.py > $O/prof.log 2>&1 || exit $?
