# ODE integrator PMC at bench sizes (262144 points = 2 waves/SIMD): VALU and FP64 instruction
# counts (one counter pass) and kernel durations (a kernel-trace stats pass) of tools/bench_ode.py.
# Summarised by tools/summarize_ode_pmc.py into profiles/<round>/ode_pmc.json.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/odepmc; rm -rf $OUT; mkdir -p $OUT
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 --output-format csv -d $OUT/pmc -o run -- python3 tools/bench_ode.py 262144 16384 > $OUT/pmc.jsonl 2> $OUT/pmc.err || { tail -5 $OUT/pmc.err; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 tools/bench_ode.py 262144 16384 > $OUT/trace.jsonl 2> $OUT/trace.err || { tail -5 $OUT/trace.err; exit 2; }
echo done
