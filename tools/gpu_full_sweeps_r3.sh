# Round 3: the full C3 (1e7), C4 (1e8) and C5 (1e6 x 8 coherent crossings) grids and the P1
# profile sweep through the sweep CLI on ONE GPU (checkpoints in local /tmp, not merged back);
# summaries -> gpurun_out/sweeps_r3/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out/sweeps_r3
PKG=baryon-and-dark-matter-densities-from-bounce--sourced-distributed-landau--zener-transport_amd
for S in C5 P1 C3 C4; do
  rm -rf /tmp/sweep_$S
  timeout -k 10 500 python -u -m $PKG.sweep --spec $S --out /tmp/sweep_$S > gpurun_out/sweeps_r3/$S.log 2>&1 || { tail -5 gpurun_out/sweeps_r3/$S.log; exit 1; }
  tail -1 gpurun_out/sweeps_r3/$S.log
  python -c "import json,sys; d=json.load(open('/tmp/sweep_$S/summary.json')); d.pop('spec_def', None); json.dump(d, open('gpurun_out/sweeps_r3/${S}_summary.json','w'), indent=1)"
  rm -rf /tmp/sweep_$S
done
echo all-done
