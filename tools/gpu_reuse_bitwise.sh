# GPU box: full C3 (1e7) and C4 (1e8) grids through the sweep CLI, dense and with --reuse-zsums,
# then the two table.npy files compared bit for bit (np.array_equal on the raw float64 rows).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out/reuse_bitwise
PKG=baryon-and-dark-matter-densities-from-bounce--sourced-distributed-landau--zener-transport_amd
for S in C3 C4; do
  rm -rf /tmp/bw_d_$S /tmp/bw_r_$S
  timeout -k 10 500 python -u -m $PKG.sweep --spec $S --out /tmp/bw_d_$S > gpurun_out/reuse_bitwise/${S}_dense.log 2>&1 || { tail -5 gpurun_out/reuse_bitwise/${S}_dense.log; exit 1; }
  timeout -k 10 300 python -u -m $PKG.sweep --spec $S --out /tmp/bw_r_$S --reuse-zsums > gpurun_out/reuse_bitwise/${S}_reuse.log 2>&1 || { tail -5 gpurun_out/reuse_bitwise/${S}_reuse.log; exit 2; }
  timeout -k 10 300 python -c "
import json, numpy as np
a = np.load('/tmp/bw_d_$S/table.npy', mmap_mode='r'); b = np.load('/tmp/bw_r_$S/table.npy', mmap_mode='r')
same = a.shape == b.shape and all(np.array_equal(a[i:i + 10**7].view(np.uint64), b[i:i + 10**7].view(np.uint64)) for i in range(0, a.shape[0], 10**7))
d = json.loads(open('gpurun_out/reuse_bitwise/${S}_dense.log').read().strip().splitlines()[-1])
r = json.loads(open('gpurun_out/reuse_bitwise/${S}_reuse.log').read().strip().splitlines()[-1])
rec = {'spec': '$S', 'points': int(a.shape[0]), 'bit_identical_tables': bool(same),
       'dense_elapsed_s': d['elapsed_s'], 'reuse_elapsed_s': r['elapsed_s']}
print(json.dumps(rec)); open('gpurun_out/reuse_bitwise/$S.json', 'w').write(json.dumps(rec))
" || exit 3
  rm -rf /tmp/bw_d_$S /tmp/bw_r_$S
done
echo all-done
