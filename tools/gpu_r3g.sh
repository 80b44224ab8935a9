# Propagator cell-data restructure + ODE Newton A/B: GPU tests of both paths with the current
# library, the scheme A/B against the committed build (c541, same S) and the round-3-start build,
# and the variant ablations.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/r3g; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests/test_gpu_propagator.py tests/test_gpu_plugin.py tests/test_gpu_ode.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python -u tools/ab_prop_scheme.py 400000 8 5 c541 64 > $OUT/ab.jsonl 2> $OUT/ab.err || { tail -20 $OUT/ab.err; exit 2; }
timeout -k 10 300 python -u tools/ab_prop_scheme.py 400000 8 5 r3head 1000 >> $OUT/ab.jsonl 2>> $OUT/ab.err || { tail -20 $OUT/ab.err; exit 2; }
cat $OUT/ab.jsonl
timeout -k 10 300 python -u tools/ablate_prop.py 400000 5 > $OUT/ablate_prop.json 2> $OUT/ablate_prop.err || { tail -20 $OUT/ablate_prop.err; exit 3; }
cat $OUT/ablate_prop.json
timeout -k 10 500 python -u tools/ablate_ode.py 262144 3 > $OUT/ablate_ode.json 2> $OUT/ablate_ode.err || { tail -20 $OUT/ablate_ode.err; exit 4; }
cat $OUT/ablate_ode.json
