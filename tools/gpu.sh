# The one GPU-box launcher (run through gpurun from the repo root):
#
#   gpurun -- bash tools/gpu.sh tests [pytest args ...]   the -m gpu suite (or a selection), one process
#   gpurun -- bash tools/gpu.sh final                     full -m gpu suite, smoke(), the default bench line
#   gpurun -- bash tools/gpu.sh profile ROUND             rocprofv3 --kernel-trace --stats of the driver's
#                                                         bench command, the PMC passes of the headline
#                                                         kernel, profiles/ROUND summary, then the bench
#   gpurun -- bash tools/gpu.sh ode-pmc                   ODE integrator PMC + kernel trace (tools/ode_pmc_run.py)
#   gpurun -- bash tools/gpu.sh prop-pmc [N]              bounce-profile propagation PMC + kernel trace
#   gpurun -- bash tools/gpu.sh lzprop-pmc                LZ propagator PMC + kernel trace (C5 slice)
#   gpurun -- [REUSE=1] bash tools/gpu.sh sweeps [SPECS]  full grids through the sweep CLI (+ reuse bitwise)
#   gpurun -- bash tools/gpu.sh bench [bench args ...]    one bench line
#   gpurun -- bash tools/gpu.sh py SCRIPT [args ...]      any tools/ script (ablations, ODE / profile benches)
#
# Every GPU step runs under its own timeout and the steps are chained: a failure, abort or
# time limit ends the call there (tail of the step's log on stdout, output under gpurun_out/).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
cmd=${1:-tests}
shift || true
OUT=gpurun_out/$cmd
mkdir -p "$OUT"

run_tests() {  # pytest args...
  timeout -k 10 1500 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread -s "$@" \
    > "$OUT/pytest_gpu.log" 2>&1 || { tail -60 "$OUT/pytest_gpu.log"; return 1; }
  grep -E "worst|passed|failed" "$OUT/pytest_gpu.log" | tail -40
}

case "$cmd" in
  tests)
    run_tests "${@:-tests}"
    ;;
  final)
    run_tests tests || exit 1
    timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
      || { tail -20 "$OUT/smoke.log"; exit 2; }
    tail -1 "$OUT/smoke.log"
    timeout -k 10 400 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 3; }
    cut -c1-600 "$OUT/bench.json"
    ;;
  profile)
    ROUND=${1:?profile ROUND}
    rm -rf "$OUT"; mkdir -p "$OUT"
    timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
      python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench_traced.json" 2> "$OUT/bench_traced.err" \
      || { tail -5 "$OUT/bench_traced.err"; exit 2; }
    cut -c1-300 "$OUT/bench_traced.json"
    P="--points 200000 --steps 1 --warmup 0 --no-cpu-baseline --no-reuse --no-parity-spot"
    pmc() { tag=$1; shift; timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/pmc_$tag" -o run -- \
      python3 bench.py $P > "$OUT/pmc_$tag.json" 2> "$OUT/pmc_$tag.err" || { echo "pmc $tag failed"; return 1; }; }
    pmc fetch FETCH_SIZE && pmc write WRITE_SIZE && \
    pmc sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT && \
    pmc inst SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_SALU SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE GRBM_COUNT && \
    pmc mix SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_INT32 || exit 4
    # the summary in the box's copy, so the plain bench below reports this build's roofline (the
    # host re-runs tools/summarize_profile.py on the merged gpurun_out to commit profiles/ROUND)
    python3 tools/summarize_profile.py "$OUT" "$ROUND" > "$OUT/summary.log" 2>&1 || { tail "$OUT/summary.log"; exit 5; }
    timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench_plain.json" 2> "$OUT/bench_plain.err" \
      || { tail -20 "$OUT/bench_plain.err"; exit 3; }
    cut -c1-600 "$OUT/bench_plain.json"
    ;;
  ode-pmc)   # the ODE integrator's instruction mix and kernel time on tools/ode_pmc_run.py's three cases;
             # summarise with: python tools/summarize_ode_pmc.py gpurun_out/ode-pmc ROUND cases
    rm -rf "$OUT"; mkdir -p "$OUT"
    timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 \
      SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 --output-format csv -d "$OUT/pmc" -o run -- \
      python3 tools/ode_pmc_run.py > "$OUT/pmc.jsonl" 2> "$OUT/pmc.err" || { tail -5 "$OUT/pmc.err"; exit 1; }
    timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
      python3 tools/ode_pmc_run.py > "$OUT/trace.jsonl" 2> "$OUT/trace.err" || { tail -5 "$OUT/trace.err"; exit 2; }
    # the non-FP64 rest of the mix (integer, conversions, scalar, LDS), its own pass
    timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 \
      SQ_INSTS_VALU_CVT SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_TRANS_F64 --output-format csv -d "$OUT/mix" -o run -- \
      python3 tools/ode_pmc_run.py > "$OUT/mix.jsonl" 2> "$OUT/mix.err" || { tail -5 "$OUT/mix.err"; exit 3; }
    # where the wave cycles go (issue stalls vs parked vs issuing), and the clock: its own pass
    timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
      SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv \
      -d "$OUT/stall" -o run -- python3 tools/ode_pmc_run.py > "$OUT/stall.jsonl" 2> "$OUT/stall.err" \
      || { tail -5 "$OUT/stall.err"; exit 4; }
    cat "$OUT/trace.jsonl"
    ;;
  configs)   # per-config throughput (tools/bench_configs.py, all configs in one process), then one PMC pass per
             # config for its executed FP64; summarise with: python tools/summarize_configs.py gpurun_out/configs ROUND
    rm -rf "$OUT"; mkdir -p "$OUT"
    timeout -k 10 400 python3 tools/bench_configs.py > "$OUT/timed.jsonl" 2> "$OUT/timed.err" \
      || { tail -5 "$OUT/timed.err"; exit 1; }
    for c in C2 C3 C4 C5 C5_N16 C5_N32 P1 O_narrow_wash O_stiff_thermal O_riccati_mchi_sv; do
      timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 \
        SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 --output-format csv -d "$OUT/pmc_$c" -o run -- \
        python3 tools/bench_configs.py --pmc --only $c --points 100000 --ode-points 65536 > "$OUT/pmc_$c.jsonl" \
        2> "$OUT/pmc_$c.err" || { tail -5 "$OUT/pmc_$c.err"; exit 2; }
    done
    cat "$OUT/timed.jsonl" | cut -c1-300
    ;;
  prop-pmc)  # the bounce-profile propagation (tools/bench_profile.py): instruction mix per kernel + kernel trace;
             # summarise with: python tools/summarize_profile_pmc.py gpurun_out/prop-pmc ROUND
    N=${1:-1000000}
    rm -rf "$OUT"; mkdir -p "$OUT"
    timeout -k 10 300 python3 tools/bench_profile.py "$N" 3 --ab --json "$OUT/bench_traced.json" > "$OUT/bench.log" 2>&1 \
      || { tail -20 "$OUT/bench.log"; exit 1; }
    cat "$OUT/bench_traced.json"
    timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 \
      SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_SALU --output-format csv -d "$OUT/pmc" -o run -- \
      python3 tools/bench_profile.py "$N" 1 --only propagate --ab > "$OUT/pmc.json" 2> "$OUT/pmc.err" || { tail -5 "$OUT/pmc.err"; exit 2; }
    timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
      SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS --output-format csv -d "$OUT/pmc_stall" -o run -- \
      python3 tools/bench_profile.py "$N" 1 --only propagate > "$OUT/pmc_stall.json" 2> "$OUT/pmc_stall.err" \
      || { tail -5 "$OUT/pmc_stall.err"; exit 2; }
    timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
      python3 tools/bench_profile.py "$N" 3 --only propagate --ab > "$OUT/trace.json" 2> "$OUT/trace.err" || { tail -5 "$OUT/trace.err"; exit 3; }
    echo done
    ;;
  lzprop-pmc)  # the LZ propagator (lz_propagate / lz_follow kernels) on a 4e5-point C5 slice: PMC + trace;
               # summarise with: python tools/summarize_prop_pmc.py gpurun_out/lzprop-pmc ROUND
    rm -rf "$OUT"; mkdir -p "$OUT"
    timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 \
      SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 --output-format csv -d "$OUT/pmc" -o run -- \
      python3 tools/prop_only.py 400000 8 1 > "$OUT/pmc.json" 2> "$OUT/pmc.err" || { tail -5 "$OUT/pmc.err"; exit 1; }
    timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
      python3 tools/prop_only.py 400000 8 3 > "$OUT/trace.json" 2> "$OUT/trace.err" || { tail -5 "$OUT/trace.err"; exit 2; }
    cat "$OUT/trace.json"
    ;;
  sweeps)  # full grids through the sweep CLI on one GPU (default C3 C4), dense and, with REUSE=1, also
           # --reuse-zsums with the two tables compared bit for bit; summaries -> gpurun_out/sweeps/
    PKG=baryon-and-dark-matter-densities-from-bounce--sourced-distributed-landau--zener-transport_amd
    for S in ${@:-C3 C4}; do
      rm -rf "/tmp/sw_d_$S" "/tmp/sw_r_$S"
      timeout -k 10 500 python3 -u -m $PKG.sweep --spec "$S" --out "/tmp/sw_d_$S" > "$OUT/${S}_dense.log" 2>&1 \
        || { tail -5 "$OUT/${S}_dense.log"; exit 1; }
      tail -1 "$OUT/${S}_dense.log"
      python3 -c "import json; d = json.load(open('/tmp/sw_d_$S/summary.json')); d.pop('spec_def', None); \
json.dump(d, open('$OUT/${S}_summary.json', 'w'), indent=1)" || exit 2
      if [ "${REUSE:-0}" = 1 ]; then
        timeout -k 10 300 python3 -u -m $PKG.sweep --spec "$S" --out "/tmp/sw_r_$S" --reuse-zsums > "$OUT/${S}_reuse.log" 2>&1 \
          || { tail -5 "$OUT/${S}_reuse.log"; exit 3; }
        timeout -k 10 300 python3 -c "
import json, numpy as np
a = np.load('/tmp/sw_d_$S/table.npy', mmap_mode='r'); b = np.load('/tmp/sw_r_$S/table.npy', mmap_mode='r')
same = a.shape == b.shape and all(np.array_equal(a[i:i + 10**7].view(np.uint64), b[i:i + 10**7].view(np.uint64))
                                  for i in range(0, a.shape[0], 10**7))
d = json.loads(open('$OUT/${S}_dense.log').read().strip().splitlines()[-1])
r = json.loads(open('$OUT/${S}_reuse.log').read().strip().splitlines()[-1])
rec = {'spec': '$S', 'points': int(a.shape[0]), 'bit_identical_tables': bool(same),
       'dense_elapsed_s': d['elapsed_s'], 'reuse_elapsed_s': r['elapsed_s']}
print(json.dumps(rec)); open('$OUT/${S}_reuse_bitwise.json', 'w').write(json.dumps(rec))" || exit 4
      fi
      rm -rf "/tmp/sw_d_$S" "/tmp/sw_r_$S"
    done
    ;;
  bench)
    timeout -k 10 600 python3 -u bench.py "$@" > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 3; }
    cut -c1-800 "$OUT/bench.json"
    ;;
  py)
    script=${1:?py SCRIPT}
    shift
    timeout -k 10 1100 python3 -u "$script" "$@" > "$OUT/$(basename "$script" .py).log" 2>&1 \
      || { tail -40 "$OUT/$(basename "$script" .py).log"; exit 6; }
    tail -40 "$OUT/$(basename "$script" .py).log"
    ;;
  *)
    echo "usage: tools/gpu.sh tests|final|profile ROUND|ode-pmc|configs|prop-pmc|lzprop-pmc|sweeps|bench|py SCRIPT ..."; exit 64
    ;;
esac
