# Tuning session: correctness, variant A/B in one process, then the plain bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/tune
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q -s --timeout 150 --timeout-method thread -m gpu tests/ > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
grep -E "worst|passed" $OUT/pytest_gpu.log
timeout -k 10 300 python -u tools/ablate_builds.py 100000 3 > $OUT/ablate_builds.json 2> $OUT/ablate_builds.err || { tail -5 $OUT/ablate_builds.err; exit 2; }
cat $OUT/ablate_builds.json
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit 3
cut -c1-400 $OUT/bench.json
