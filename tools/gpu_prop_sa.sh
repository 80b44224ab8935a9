# Superadiabatic-following propagator: GPU tests that touch lzq_lz_propagate, the scheme A/B
# (vs the round-3 HEAD build in _build/variants) at 8/16/32 crossings, and a kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/propsa; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_propagator.py tests/test_gpu_plugin.py tests/test_gpu_configs.py tests/test_gpu_sweep.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for nc in 8 16 32; do
  timeout -k 10 300 python -u tools/ab_prop_scheme.py 400000 $nc 5 >> $OUT/ab.jsonl 2>> $OUT/ab.err || { tail -20 $OUT/ab.err; exit 2; }
done
cat $OUT/ab.jsonl
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 tools/prop_only.py 400000 8 3 > $OUT/trace.json 2> $OUT/trace.err || { tail -5 $OUT/trace.err; exit 3; }
cat $OUT/trace.json
echo done
