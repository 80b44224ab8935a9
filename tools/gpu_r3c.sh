# Profile-propagator PMC + kernel trace (1e6 points), then the ODE throughput bench (sub-groups)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/profprop; mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 --output-format csv -d $OUT/pmc -o run -- python3 tools/bench_profile.py 1000000 1 --only propagate > $OUT/pmc.json 2> $OUT/pmc.err || { tail -5 $OUT/pmc.err; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 tools/bench_profile.py 1000000 3 --json $OUT/bench_traced.json > $OUT/trace.json 2> $OUT/trace.err || { tail -5 $OUT/trace.err; exit 2; }
cat $OUT/bench_traced.json
mkdir -p gpurun_out/ode
timeout -k 10 600 python3 tools/bench_ode.py 262144 2048 > gpurun_out/ode/bench_ode.jsonl 2> gpurun_out/ode/bench_ode.err || { tail -20 gpurun_out/ode/bench_ode.err; exit 3; }
cat gpurun_out/ode/bench_ode.jsonl
echo done
