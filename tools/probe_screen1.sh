# One-limb pass timing probes (tools/probe/screen1_probe.hip), built on the CPU
# side into tools/bin/: the previous kernel (screen1_old) beside the current
# one and its probe modes.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && for b in ${PROBES:-old m0 m2}; do timeout -k 5 120 ./tools/bin/screen1_$b || exit 1; done
