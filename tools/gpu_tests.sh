# GPU test suite only.  Usage: bash tools/gpu_tests.sh <tag> [pytest -k expr]
set -o pipefail
R=$GRAFT_REPO_ROOT; T=${1:-tests}; O=$R/gpurun_out/$T
mkdir -p $O && cd $R
K=${2:+-k "$2"}
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread $K > $O/pytest_gpu.log 2>&1; rc=$?
tail -30 $O/pytest_gpu.log
exit $rc
