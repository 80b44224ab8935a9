# GPU box: the full -m gpu suite (one pytest process), smoke, and the counter list of this
# rocprofv3 (for choosing PMC passes).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out/t
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -s > gpurun_out/t/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/t/pytest_gpu.log; exit 1; }
grep -E "worst|passed|failed" gpurun_out/t/pytest_gpu.log | tail -12
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/t/smoke.log 2>&1 || { tail -20 gpurun_out/t/smoke.log; exit 2; }
tail -1 gpurun_out/t/smoke.log
if [ -n "$LIST_COUNTERS" ]; then timeout -k 10 120 rocprofv3 -L > gpurun_out/t/counters.txt 2>&1 || echo "counter list failed"; fi
echo done
