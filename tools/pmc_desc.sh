bash tools/pmc_kernel.sh "blur_octave" blur --batch 16
