# Round profile: full bench (with CPU baseline), rocprofv3 kernel trace + stats, PMC passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/prof
mkdir -p $OUT
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
timeout -k 10 300 python -u bench.py > $OUT/bench_full.json 2> $OUT/bench_full.err || exit 2
cat $OUT/bench_full.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --points 200000 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/trace_bench.json 2> $OUT/trace.err || exit 3
for c in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"; do
  tag=$(echo $c | cut -d' ' -f1)
  timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d $OUT/pmc_$tag -o run -- python3 bench.py --points 200000 --steps 1 --warmup 0 --no-cpu-baseline > $OUT/pmc_$tag.json 2> $OUT/pmc_$tag.err || { echo "pmc $tag failed"; tail -3 $OUT/pmc_$tag.err; }
done
find $OUT -name '*.csv' | head -50
