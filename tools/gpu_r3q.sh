# One-point ODE latency (the CLI's case) after the linear integrator variant.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/r3q; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 300 python -u tools/time_ode_single.py > $OUT/time_ode_single.jsonl 2> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
cat $OUT/time_ode_single.jsonl
