# Round profile: the default bench command under rocprofv3 --kernel-trace --stats (so the
# committed kernel stats describe the same command as BENCH), then PMC passes (one counter
# group per run; FETCH_SIZE and WRITE_SIZE separate, per MI355X_MICROARCH.md) on a smaller grid.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/prof
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_traced.json 2> $OUT/bench_traced.err || { tail -5 $OUT/bench_traced.err; exit 2; }
cat $OUT/bench_traced.json
P="--points 200000 --steps 1 --warmup 0 --no-cpu-baseline --no-reuse --no-parity-spot"
pmc() { tag=$1; shift; timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $OUT/pmc_$tag -o run -- python3 bench.py $P > $OUT/pmc_$tag.json 2> $OUT/pmc_$tag.err || echo "pmc $tag failed"; }
pmc fetch FETCH_SIZE
pmc write WRITE_SIZE
pmc sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT
pmc inst SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_SALU SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE GRBM_COUNT
pmc mix SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_INT32
# refresh profiles/round3/pmc_summary.json in the box's copy, so the plain bench's roofline
# fields come from this build's counters (the host re-runs the summary on the merged output)
python3 tools/summarize_profile.py $OUT round3 > $OUT/summary.log 2>&1 || echo "summary failed"
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_plain.json 2> $OUT/bench_plain.err || exit 3
cat $OUT/bench_plain.json
echo done
