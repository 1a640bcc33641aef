bash tools/pmc_kernel.sh "descriptor" desc3 --batch 16
