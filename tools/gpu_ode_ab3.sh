# ODE A/B (tools/ablate_ode.py on the variants under _build/variants) + ODE PMC of the default build
# on the m_chi x sigma_v sweep
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/odeab; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 600 python3 tools/ablate_ode.py 262144 3 > $OUT/ablate.json 2> $OUT/ablate.err || { tail -20 $OUT/ablate.err; exit 1; }
cat $OUT/ablate.json
echo done
