#!/bin/bash
# Kernel trace of tools/prop_only.py (4e5 C5 points x 8 crossings) for every library variant under
# <package>/_build/variants/: lz_follow_kernel / lz_propagate_kernel average durations per variant.
#   gpurun -- bash tools/ablate_follow.sh
set -o pipefail
OUT=gpurun_out/ablate_follow
rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
for so in baryon-and-dark-matter-densities-from-bounce--sourced-distributed-landau--zener-transport_amd/_build/variants/*.so; do
  name=$(basename "$so" .so)
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$name" -o run -- \
    python3 tools/prop_only.py 400000 8 5 "$so" > "$OUT/$name.json" 2> "$OUT/$name.err" || { tail -5 "$OUT/$name.err"; exit 1; }
  f=$(find "$OUT/$name" -name "*kernel_stats.csv" | head -1)
  echo "$name $(cat "$OUT/$name.json")"
  grep -E "lz_follow|lz_propagate_kernel" "$f" | cut -d, -f1-6
done
