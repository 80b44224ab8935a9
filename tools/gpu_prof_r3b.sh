# Profile path: bench (random and v_w-ordered launch, 1e5 and 1e6 points), variant ablation, tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/profprop; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 200 python3 tools/bench_profile.py 100000 3 --json $OUT/bench.json > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
timeout -k 10 200 python3 tools/bench_profile.py 100000 3 --sort-vw --json $OUT/bench_sorted.json > $OUT/bench_sorted.log 2>&1 || exit 2
timeout -k 10 200 python3 tools/bench_profile.py 1000000 3 --json $OUT/bench_1e6.json > $OUT/bench_1e6.log 2>&1 || exit 3
timeout -k 10 200 python3 tools/bench_profile.py 1000000 3 --sort-vw --json $OUT/bench_1e6_sorted.json > $OUT/bench_1e6s.log 2>&1 || exit 4
cat $OUT/bench*.json
timeout -k 10 300 python3 tools/ablate_profile.py 1000000 5 > $OUT/ablate.json 2> $OUT/ablate.err || { tail -5 $OUT/ablate.err; exit 5; }
cat $OUT/ablate.json
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 --output-format csv -d $OUT/pmc -o run -- python3 tools/bench_profile.py 1000000 1 --only propagate > $OUT/pmc.json 2> $OUT/pmc.err || { tail -5 $OUT/pmc.err; exit 6; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 tools/bench_profile.py 1000000 3 > $OUT/trace.json 2> $OUT/trace.err || { tail -5 $OUT/trace.err; exit 7; }
echo done
