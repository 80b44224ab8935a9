# Round 3 (session 2) validation at HEAD: full -m gpu suite, smoke, propagator PMC, bench, ODE PMC.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
bash tools/gpu_r3e.sh || exit $?
bash tools/gpu_ode_pmc3.sh || exit 6
mkdir -p gpurun_out/cfg
timeout -k 10 400 python -u tools/bench_configs.py 400000 > gpurun_out/cfg/bench_configs.jsonl 2> gpurun_out/cfg/bench_configs.err || { tail -20 gpurun_out/cfg/bench_configs.err; exit 7; }
cut -c1-200 gpurun_out/cfg/bench_configs.jsonl
