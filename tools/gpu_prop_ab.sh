# GPU box: propagator tests, then the A/B of the library variants under _build/variants
# (tools/ablate_prop.py: one process, interleaved rounds, bit-identity across variants), then
# a kernel trace of the default build's C5 propagator (cost / scan / scatter / propagate).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out/prop
timeout -k 10 300 python -u -m pytest tests/test_gpu_propagator.py -x -v --timeout 120 --timeout-method thread > gpurun_out/prop/pytest.log 2>&1 || { tail -30 gpurun_out/prop/pytest.log; exit 1; }
tail -2 gpurun_out/prop/pytest.log
timeout -k 10 300 python -u tools/ablate_prop.py 400000 5 > gpurun_out/prop/ablate.json 2>&1 || { cat gpurun_out/prop/ablate.json; exit 2; }
cat gpurun_out/prop/ablate.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prop/trace -o run -- python3 tools/prop_only.py 400000 8 3 > gpurun_out/prop/prop_only.json 2>&1 || { tail -5 gpurun_out/prop/prop_only.json; exit 3; }
tail -1 gpurun_out/prop/prop_only.json
echo done
