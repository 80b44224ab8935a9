# Host-side record transfer without the extra copy: the GPU tests that go through
# points_to_device / Engine.ode / profile_points, and bench_ode.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/r3l; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests/test_gpu_ode.py tests/test_gpu_cli.py tests/test_gpu_plugin.py tests/test_gpu_profile.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 600 python -u tools/bench_ode.py 262144 16384 > $OUT/bench_ode.jsonl 2> $OUT/bench_ode.err || { tail -20 $OUT/bench_ode.err; exit 3; }
cut -c1-330 $OUT/bench_ode.jsonl
