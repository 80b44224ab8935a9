# Propagator PMC: VALU / FP64 instruction counts and kernel time of lz_propagate_kernel on a
# 4e5-point C5 slice (tools/prop_only.py), one counter pass + one kernel-trace pass.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/proppmc; rm -rf $OUT; mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 --output-format csv -d $OUT/pmc -o run -- python3 tools/prop_only.py 400000 8 1 > $OUT/pmc.json 2> $OUT/pmc.err || { tail -5 $OUT/pmc.err; exit 1; }
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 tools/prop_only.py 400000 8 3 > $OUT/trace.json 2> $OUT/trace.err || { tail -5 $OUT/trace.err; exit 2; }
cat $OUT/trace.json
echo done
