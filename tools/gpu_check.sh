# GPU correctness + quick perf check (used during development).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 150 --timeout-method thread -m gpu tests/ > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"
grep -E "passed|failed|worst" gpurun_out/pytest_gpu.log | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 3
tail -1 gpurun_out/smoke.log
timeout -k 10 200 python -u tools/ablate_exp.py 200000 3 > gpurun_out/ablate.log 2>&1 || exit 4
cat gpurun_out/ablate.log
