bash tools/pmc_kernel.sh "descriptor" v2 --batch 8 && SIFT_HIP_DESC_V1=1 bash tools/pmc_kernel.sh "descriptor" v1 --batch 8
