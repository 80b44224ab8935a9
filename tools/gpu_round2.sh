# GPU box: -m gpu suite, then the round profile (tools/gpu_profile.sh), then the ODE throughput.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
bash tools/gpu_tests.sh || exit 1
bash tools/gpu_profile.sh || exit 2
mkdir -p gpurun_out/ode
timeout -k 10 400 python -u tools/bench_ode.py 262144 131072 > gpurun_out/ode/bench_ode.jsonl 2> gpurun_out/ode/bench_ode.err || { tail -20 gpurun_out/ode/bench_ode.err; exit 3; }
cat gpurun_out/ode/bench_ode.jsonl
echo all-done
