# GPU box: -m gpu suite, the ODE throughput, and the ODE variant ablation (_build/variants/).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
bash tools/gpu_tests.sh || exit 1
mkdir -p gpurun_out/ode2
timeout -k 10 400 python -u tools/bench_ode.py 262144 131072 > gpurun_out/ode2/bench_ode.jsonl 2> gpurun_out/ode2/bench_ode.err || { tail -20 gpurun_out/ode2/bench_ode.err; exit 3; }
cat gpurun_out/ode2/bench_ode.jsonl
timeout -k 10 400 python -u tools/ablate_ode.py 262144 3 > gpurun_out/ode2/ablate_ode.json 2>&1 || { cat gpurun_out/ode2/ablate_ode.json; exit 5; }
cat gpurun_out/ode2/ablate_ode.json
echo all-done
