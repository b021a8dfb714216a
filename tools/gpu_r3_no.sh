# Round 3 steps N + O in one call
bash tools/gpu_r3_n.sh && bash tools/gpu_r3_o.sh
