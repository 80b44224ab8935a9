# bench_ode at the final round-3 build.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/r3s; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 600 python -u tools/bench_ode.py 262144 16384 > $OUT/bench_ode.jsonl 2> $OUT/bench_ode.err || { tail -20 $OUT/bench_ode.err; exit 1; }
cut -c1-420 $OUT/bench_ode.jsonl
