# GPU box: golden accuracy + C2 quadrature A/B + ODE A/B over every variant in _build/variants.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out/ab2
timeout -k 10 300 python -u tools/diag_golden.py > gpurun_out/ab2/diag_golden.json 2> gpurun_out/ab2/diag.err || { tail -5 gpurun_out/ab2/diag.err; exit 1; }
timeout -k 10 300 python -u tools/ablate_builds.py 200000 4 > gpurun_out/ab2/ablate_c2.json 2>&1 || { cat gpurun_out/ab2/ablate_c2.json; exit 2; }
cat gpurun_out/ab2/ablate_c2.json
timeout -k 10 400 python -u tools/ablate_ode.py 262144 3 > gpurun_out/ab2/ablate_ode.json 2>&1 || { cat gpurun_out/ab2/ablate_ode.json; exit 3; }
cat gpurun_out/ab2/ablate_ode.json
echo all-done
