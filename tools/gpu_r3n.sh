# ODE linear waves in their own kernel variant (tight loop per block): ODE GPU tests, A/B, bench_ode.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/r3n; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_ode.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 500 python -u tools/ablate_ode.py 262144 3 > $OUT/ablate_ode.json 2> $OUT/ablate_ode.err || { tail -20 $OUT/ablate_ode.err; exit 2; }
cat $OUT/ablate_ode.json
timeout -k 10 600 python -u tools/bench_ode.py 262144 16384 > $OUT/bench_ode.jsonl 2> $OUT/bench_ode.err || { tail -20 $OUT/bench_ode.err; exit 3; }
cut -c1-300 $OUT/bench_ode.jsonl
