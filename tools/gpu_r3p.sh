# ODE predictor as an fma chain: the ODE GPU tests and the one-process A/B (262,144 points,
# one chunk) against the previous build.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/r3p; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_ode.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 500 python -u tools/ablate_ode.py 262144 3 > $OUT/ablate_ode.json 2> $OUT/ablate_ode.err || { tail -20 $OUT/ablate_ode.err; exit 2; }
cat $OUT/ablate_ode.json
