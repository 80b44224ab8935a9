set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out/ab
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab/pytest.log 2>&1 || { tail -30 gpurun_out/ab/pytest.log; exit 1; }
tail -3 gpurun_out/ab/pytest.log
timeout -k 10 300 python tools/ablate_builds.py 200000 4 > gpurun_out/ab/ablate.json 2>&1 || { cat gpurun_out/ab/ablate.json; exit 2; }
cat gpurun_out/ab/ablate.json
P="--points 200000 --steps 1 --warmup 0 --no-cpu-baseline"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/ab/pmc_fetch -o run -- python3 bench.py $P > gpurun_out/ab/pmc_fetch.json 2>&1 || echo fetch failed
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/ab/pmc_write -o run -- python3 bench.py $P > gpurun_out/ab/pmc_write.json 2>&1 || echo write failed
echo done
