for d in 55 119 183 247; do echo "== dbg=$d"; PBX_ATTN_DBG=$d timeout -k 10 100 python tools/kbench_attn.py 2>&1 | grep "WG dur"; done
