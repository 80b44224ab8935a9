# Reflection-symmetric core-edge frames in lz_follow_kernel: propagator GPU tests and the A/B
# against the previous commit (same S) and the round-3-start build.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/r3i; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_propagator.py tests/test_gpu_plugin.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for nc in 8 16 32; do
timeout -k 10 300 python -u tools/ab_prop_scheme.py 400000 $nc 7 prerefl 64 >> $OUT/ab.jsonl 2>> $OUT/ab.err || { tail -20 $OUT/ab.err; exit 2; }
done
timeout -k 10 300 python -u tools/ab_prop_scheme.py 400000 8 7 r3head 1000 >> $OUT/ab.jsonl 2>> $OUT/ab.err || { tail -20 $OUT/ab.err; exit 2; }
cat $OUT/ab.jsonl
bash tools/gpu_prop_pmc.sh
