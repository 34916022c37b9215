timeout -k 10 60 tools/lab/skinny_trace 11008 4096 32 > gpurun_out/sk_trace.log 2>&1 && bash tools/pmc_sq.sh tools/lab/skinny_trace gemm_skinny > gpurun_out/sk_pmc.txt 2>&1
