# GPU box: the full C3 (1e7) and C4 (1e8) grids through the sweep CLI with --reuse-zsums (the
# z-sums shared per y-grid / A/V kernel; not the headline mode), checkpointing to local /tmp;
# the grid statistics must equal those of the dense runs of tools/gpu_full_sweeps.sh (run first,
# same build) exactly (bit-identical
# tables reduce to the same numbers).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out/sweeps_reuse
PKG=baryon-and-dark-matter-densities-from-bounce--sourced-distributed-landau--zener-transport_amd
for S in C3 C4; do
  rm -rf /tmp/sweepr_$S
  timeout -k 10 500 python -u -m $PKG.sweep --spec $S --out /tmp/sweepr_$S --reuse-zsums > gpurun_out/sweeps_reuse/$S.log 2>&1 || { tail -5 gpurun_out/sweeps_reuse/$S.log; exit 1; }
  tail -1 gpurun_out/sweeps_reuse/$S.log
  python -c "
import json
d = json.load(open('/tmp/sweepr_$S/summary.json')); d.pop('spec_def')
ref = json.load(open('gpurun_out/sweeps/${S}_summary.json'))
d['final_equals_dense_run'] = d['final'] == ref['final']
json.dump(d, open('gpurun_out/sweeps_reuse/${S}_summary.json', 'w'), indent=1)
print('$S final stats equal to the dense run:', d['final_equals_dense_run'])"
  rm -rf /tmp/sweepr_$S
done
echo all-done
