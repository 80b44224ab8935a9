# Tuning session: correctness, variant A/B in one process, PMC stall counters.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/tune
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/ > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -u tools/ablate_builds.py 100000 3 > $OUT/ablate_builds.json 2> $OUT/ablate_builds.err || { tail -5 $OUT/ablate_builds.err; exit 2; }
cat $OUT/ablate_builds.json
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $OUT/pmc_stall -o run -- python3 bench.py --points 100000 --steps 1 --warmup 0 --no-cpu-baseline > /dev/null 2> $OUT/pmc_stall.err || echo "pmc stall failed"
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $OUT/pmc_inst -o run -- python3 bench.py --points 100000 --steps 1 --warmup 0 --no-cpu-baseline > /dev/null 2> $OUT/pmc_inst.err || echo "pmc inst failed"
echo done
