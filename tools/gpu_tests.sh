# GPU test suite only.  Usage: bash tools/gpu_tests.sh <tag> [pytest -k expr]
set -o pipefail
R=$GRAFT_REPO_ROOT; T=${1:-tests}; O=$R/gpurun_out/$T
mkdir -p $O && cd $R
K=()
if [ -n "$2" ]; then K=(-k "$2"); fi
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread "${K[@]}" > $O/pytest_sel.log 2>&1; rc=$?
tail -30 $O/pytest_sel.log
exit $rc
