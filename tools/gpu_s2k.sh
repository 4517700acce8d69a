# A/B: streaming vs plain accesses in the headline kernel (alternating, 3 runs each) + short-line parity.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/s2k
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_short_lines.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
for r in 1 2 3; do
  timeout -k 10 200 python -u tools/ab_nt.py nt > $O/nt_$r.log 2>&1 || exit $?
  timeout -k 10 200 python -u tools/ab_nt.py nont > $O/nont_$r.log 2>&1 || exit $?
done
