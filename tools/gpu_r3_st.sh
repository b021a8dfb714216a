# Round 3 steps V + S + U + T in one call
bash tools/gpu_r3_v.sh && bash tools/gpu_r3_s.sh && bash tools/gpu_r3_u.sh && bash tools/gpu_r3_t.sh
