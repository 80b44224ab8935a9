# GPU box: -m gpu suite, ODE throughput, then the variant ablations (propagator core on/off,
# ODE integrator waves/SIMD) from <pkg>/_build/variants/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
bash tools/gpu_tests.sh || exit 1
mkdir -p gpurun_out/ab2
timeout -k 10 400 python -u tools/bench_ode.py 262144 131072 > gpurun_out/ab2/bench_ode.jsonl 2> gpurun_out/ab2/bench_ode.err || { tail -20 gpurun_out/ab2/bench_ode.err; exit 3; }
cat gpurun_out/ab2/bench_ode.jsonl
timeout -k 10 300 python -u tools/ablate_prop.py 400000 3 > gpurun_out/ab2/ablate_prop.json 2>&1 || { cat gpurun_out/ab2/ablate_prop.json; exit 4; }
cat gpurun_out/ab2/ablate_prop.json
timeout -k 10 400 python -u tools/ablate_ode.py 262144 3 > gpurun_out/ab2/ablate_ode.json 2>&1 || { cat gpurun_out/ab2/ablate_ode.json; exit 5; }
cat gpurun_out/ab2/ablate_ode.json
echo all-done
