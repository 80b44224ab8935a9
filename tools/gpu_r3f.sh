# Round 3 (session 2): full -m gpu suite + smoke (committed library), propagator PMC, bench, then
# the ODE Newton A/B variants (tools/ablate_ode.py over _build/variants).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
bash tools/gpu_r3e.sh || exit $?
mkdir -p gpurun_out/odeab
timeout -k 10 400 python -u tools/ablate_ode.py 262144 3 > gpurun_out/odeab/ablate_ode.json 2> gpurun_out/odeab/ablate_ode.err || { tail -20 gpurun_out/odeab/ablate_ode.err; exit 5; }
cat gpurun_out/odeab/ablate_ode.json
