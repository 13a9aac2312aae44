set -u
bash tools/pmc.sh top gpurun_out/pmc_h2 fwd --bf16 && cat gpurun_out/pmc_h2/summary.txt | head -40
PU_CONV_HALO=1 bash tools/pmc.sh top gpurun_out/pmc_h1 fwd --bf16 && cat gpurun_out/pmc_h1/summary.txt | head -40
