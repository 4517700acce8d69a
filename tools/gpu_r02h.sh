set -o pipefail
O=gpurun_out/r02h
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_nc_mirror.py tests/test_cpp_shim.py > $O/pytest_ncm.log 2>&1 || exit $?
