# GPU box: full GPU test suite, smoke, then the ODE-fallback throughput (profiles/round1/bench_ode.jsonl).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out/round
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/round/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/round/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/round/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/round/smoke.log 2>&1 || { tail -20 gpurun_out/round/smoke.log; exit 2; }
tail -1 gpurun_out/round/smoke.log
timeout -k 10 400 python -u tools/bench_ode.py 262144 131072 > gpurun_out/round/bench_ode.jsonl 2> gpurun_out/round/bench_ode.err || { tail -20 gpurun_out/round/bench_ode.err; exit 3; }
cat gpurun_out/round/bench_ode.jsonl
echo done
