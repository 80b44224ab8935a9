# Round 3 (session 2) first GPU call: the full -m gpu suite and smoke at HEAD, then the ODE PMC.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out/t
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -s > gpurun_out/t/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/t/pytest_gpu.log; exit 1; }
grep -E "passed|failed" gpurun_out/t/pytest_gpu.log | tail -3
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/t/smoke.log 2>&1 || { tail -20 gpurun_out/t/smoke.log; exit 2; }
tail -1 gpurun_out/t/smoke.log
bash tools/gpu_ode_pmc3.sh
