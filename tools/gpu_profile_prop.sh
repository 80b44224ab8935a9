# Bounce-profile path on one MI355X: tools/bench_profile.py (1e5 points x 16 shapes x 256 knots),
# then lzq_lz_propagate_profile alone under rocprofv3: one PMC pass (VALU / FP64 instruction
# mix) and one --kernel-trace --stats pass.  -> gpurun_out/profprop
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/profprop; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 200 python3 tools/bench_profile.py 100000 3 --json $OUT/bench.json > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
cat $OUT/bench.json
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 --output-format csv -d $OUT/pmc -o run -- python3 tools/bench_profile.py 100000 1 --only propagate > $OUT/pmc.json 2> $OUT/pmc.err || { tail -5 $OUT/pmc.err; exit 2; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 tools/bench_profile.py 100000 3 > $OUT/trace.json 2> $OUT/trace.err || { tail -5 $OUT/trace.err; exit 3; }
echo done
