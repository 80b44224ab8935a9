# Round 3 (session 2): full -m gpu suite and smoke after the propagator rework, the propagator
# PMC, and the default bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out/t
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -s > gpurun_out/t/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/t/pytest_gpu.log; exit 1; }
grep -E "passed|failed" gpurun_out/t/pytest_gpu.log | tail -2
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/t/smoke.log 2>&1 || { tail -20 gpurun_out/t/smoke.log; exit 2; }
tail -1 gpurun_out/t/smoke.log
bash tools/gpu_prop_pmc.sh || exit 3
timeout -k 10 300 python -u bench.py > gpurun_out/t/bench.json 2> gpurun_out/t/bench.err || { tail -20 gpurun_out/t/bench.err; exit 4; }
cat gpurun_out/t/bench.json
