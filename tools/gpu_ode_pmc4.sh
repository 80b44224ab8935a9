# ODE integrator PMC after the linear-wave kernel variant (round 3): tools/ode_pmc_run.py three 262,144-point
# wash-out, stiff thermal, the verdict's m_chi x sigma_v Riccati sweep), one counter pass and
# one kernel-trace pass; summarise with `tools/summarize_ode_pmc.py gpurun_out/odepmc4 round3 cases`.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/odepmc4; rm -rf $OUT; mkdir -p $OUT
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 --output-format csv -d $OUT/pmc -o run -- python3 tools/ode_pmc_run.py > $OUT/pmc.jsonl 2> $OUT/pmc.err || { tail -5 $OUT/pmc.err; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 tools/ode_pmc_run.py > $OUT/trace.jsonl 2> $OUT/trace.err || { tail -5 $OUT/trace.err; exit 2; }
cat $OUT/trace.jsonl
echo done
cp $OUT/trace/run_kernel_stats.csv $OUT/kernel_stats.csv 2>/dev/null; true
