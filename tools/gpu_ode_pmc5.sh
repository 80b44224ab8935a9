# ODE integrator stall counters (round 3): tools/ode_pmc_run.py's three cases, one pass of
# wave-cycle / wait / active-instruction counters; summarised by hand into profiles/round3.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/odepmc5; rm -rf $OUT; mkdir -p $OUT
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU --output-format csv -d $OUT/pmc -o run -- python3 tools/ode_pmc_run.py > $OUT/pmc.jsonl 2> $OUT/pmc.err || { tail -5 $OUT/pmc.err; exit 1; }
echo done
