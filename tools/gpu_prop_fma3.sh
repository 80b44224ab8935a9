# A/B of the three-address fma in cos_sinc and of the Magnus unroll (tools/build_variants.py
# LZQ_SU2_FMA3 / LZQ_PROP_UNROLL), on the C5 propagator and the profile propagator.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/fma3; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 300 python -u tools/ablate_prop.py 400000 5 > $OUT/ablate_prop.json 2> $OUT/ablate_prop.err || { tail -20 $OUT/ablate_prop.err; exit 1; }
cat $OUT/ablate_prop.json
timeout -k 10 300 python -u tools/ablate_profile.py 1000000 3 > $OUT/ablate_profile.json 2> $OUT/ablate_profile.err || { tail -20 $OUT/ablate_profile.err; exit 2; }
cat $OUT/ablate_profile.json
echo done
