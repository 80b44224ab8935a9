set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 150 --timeout-method thread -m gpu tests/ > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"
tail -5 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 3
cat gpurun_out/smoke.log
timeout -k 10 200 python -u bench.py --points 200000 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_small.log 2>&1 || exit 4
cat gpurun_out/bench_small.log
