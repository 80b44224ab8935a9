# GPU box: ODE tests, the cooperative-mode A/B (tools/ablate_ode.py over _build/variants), and
# the ODE throughput table (tools/bench_ode.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out/ode3
timeout -k 10 300 python -u -m pytest tests/test_gpu_ode.py -x -v -s --timeout 200 --timeout-method thread > gpurun_out/ode3/pytest.log 2>&1 || { tail -40 gpurun_out/ode3/pytest.log; exit 1; }
tail -2 gpurun_out/ode3/pytest.log
timeout -k 10 400 python -u tools/ablate_ode.py 262144 3 > gpurun_out/ode3/ablate_ode.json 2>&1 || { cat gpurun_out/ode3/ablate_ode.json; exit 2; }
cat gpurun_out/ode3/ablate_ode.json
timeout -k 10 400 python -u tools/bench_ode.py 262144 131072 > gpurun_out/ode3/bench_ode.jsonl 2> gpurun_out/ode3/bench_ode.err || { tail -20 gpurun_out/ode3/bench_ode.err; exit 3; }
cat gpurun_out/ode3/bench_ode.jsonl
echo all-done
