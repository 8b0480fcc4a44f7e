# Multinomial margins timing probes (tools/probe/mlr_probe.hip, built on the
# CPU side into tools/bin/mlr_m<bits>).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && for b in ${PROBES:-m0 m1 m2 m4 m3 m7}; do timeout -k 5 120 ./tools/bin/mlr_$b || exit 1; done
