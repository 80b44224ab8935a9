# GPU box: a selection of the -m gpu suite (one pytest process).  Usage: tools/gpu_tests_sel.sh <pytest args...>
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out/t
timeout -k 10 900 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread -s "$@" > gpurun_out/t/pytest_sel.log 2>&1 || { tail -60 gpurun_out/t/pytest_sel.log; exit 1; }
grep -E "worst|passed|failed|PASSED|FAILED" gpurun_out/t/pytest_sel.log | tail -40
