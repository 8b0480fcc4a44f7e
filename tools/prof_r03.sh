# Round-3 closing profiles: rocprofv3 kernel stats + FETCH/WRITE passes for
# KMeans and the Gramian, SQ passes over the KMeans kernels.
cd $GRAFT_REPO_ROOT
bash tools/prof.sh r03c_kmeans --workload kmeans --steps 5 --warmup 2 && echo KM_PROF_OK && \
bash tools/prof.sh r03c_gramian --workload gramian --steps 2 --warmup 1 && echo GRAM_PROF_OK && \
bash tools/pmc_mfma.sh kmeans 'k_screen32|k_chunk_sums|k_screen_cands' --workload kmeans > gpurun_out/pmc_kmeans.txt && echo KM_PMC_OK
