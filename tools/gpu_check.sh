# GPU correctness + quick perf check (used during development).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v -s --timeout 150 --timeout-method thread -m gpu tests/ > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"
grep -E "passed|failed|worst|Error|assert" gpurun_out/pytest_gpu.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 3
tail -1 gpurun_out/smoke.log
# rehearse the N>1 bench path (2 ranks sharing the one GPU, gloo for the gather)
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 1 --warmup 1 --points 20000 --dist-backend gloo > gpurun_out/bench_2rank.log 2>&1 || { tail -20 gpurun_out/bench_2rank.log; exit 5; }
grep metric gpurun_out/bench_2rank.log | cut -c1-300
