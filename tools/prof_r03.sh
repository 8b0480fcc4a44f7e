cd $GRAFT_REPO_ROOT
bash tools/prof.sh r03b_kmeans --workload kmeans --steps 5 --warmup 2 && echo KM_PROF_OK && \
bash tools/prof.sh r03b_lr_multi --workload lr_multi --steps 3 --warmup 1 && echo MLR_PROF_OK && \
bash tools/pmc_mfma.sh kmeans 'k_screen32|k_chunk_sums' --workload kmeans > gpurun_out/pmc_kmeans.txt && echo KM_PMC_OK && \
bash tools/pmc_mfma.sh lr_multi 'k_mlr' --workload lr_multi > gpurun_out/pmc_lr_multi.txt && echo MLR_PMC_OK && \
bash tools/pmc_mfma.sh lr_sparse 'k_tiles' --workload lr_sparse > gpurun_out/pmc_lr_sparse.txt && echo SP_PMC_OK
