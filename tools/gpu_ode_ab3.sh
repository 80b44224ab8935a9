# ODE A/B (tools/ablate_ode.py on the variants under _build/variants), then the ODE GPU tests of
# the default build
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/odeab; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 600 python3 tools/ablate_ode.py 262144 3 > $OUT/ablate.json 2> $OUT/ablate.err || { tail -20 $OUT/ablate.err; exit 1; }
cat $OUT/ablate.json
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ode.py > $OUT/pytest_ode.log 2>&1 || { tail -30 $OUT/pytest_ode.log; exit 1; }
tail -3 $OUT/pytest_ode.log
echo done
