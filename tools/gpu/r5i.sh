# full GPU suite on the final round-4 tree
set -u
O=gpurun_out/r5i; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/suite.log 2>&1; rc=$?
echo "suite rc=$rc"; tail -2 $O/suite.log; exit $rc
