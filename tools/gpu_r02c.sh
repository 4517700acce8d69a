set -o pipefail
O=gpurun_out/r02c
mkdir -p $O
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o run -- python3 $R/tools/prof_refresh.py > $R/$O/prof_refresh.log 2>&1 || exit $?
