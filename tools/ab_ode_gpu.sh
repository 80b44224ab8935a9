# GPU box: ODE variant ablation (tools/ablate_ode.py) after the GPU test suite, plus one PMC
# pass of the FP64/INT32 VALU instruction counters on the quadrature bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out/abo
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/abo/pytest.log 2>&1 || { tail -30 gpurun_out/abo/pytest.log; exit 1; }
tail -2 gpurun_out/abo/pytest.log
timeout -k 10 400 python tools/ablate_ode.py 65536 3 > gpurun_out/abo/ablate.json 2>&1 || { cat gpurun_out/abo/ablate.json; exit 2; }
cat gpurun_out/abo/ablate.json
P="--points 200000 --steps 1 --warmup 0 --no-cpu-baseline"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_INT32 --output-format csv -d gpurun_out/abo/pmc_f64 -o run -- python3 bench.py $P > gpurun_out/abo/pmc_f64.json 2> gpurun_out/abo/pmc_f64.err || { echo f64 pass failed; tail -3 gpurun_out/abo/pmc_f64.err; }
echo done
