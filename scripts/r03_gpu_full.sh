# the whole GPU suite on this tree (log under gpurun_out/)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03_pytest_full.log 2>&1; rc=$?
tail -3 gpurun_out/r03_pytest_full.log
[ $rc -ne 0 ] && grep -E "^FAILED|^E  " gpurun_out/r03_pytest_full.log | head -30
exit $rc
