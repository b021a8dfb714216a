# Round 3 steps Q + R + S in one call
bash tools/gpu_r3_q.sh && bash tools/gpu_r3_r.sh && bash tools/gpu_r3_s.sh
