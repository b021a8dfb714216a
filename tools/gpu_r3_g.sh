# Round 3 step G: same-box A/B of the GELU core rewrite (old = HEAD common.h build) with the prenorm pool
R=$GRAFT_REPO_ROOT
cd $R
T="timeout -k 10"
for i in 1 2 3; do
  $T 300 python -u bench.py > gpurun_out/r3g_new_$i.json 2> gpurun_out/r3g_new_$i.err || exit 1
  PBX_HIP_LIB=$R/tools/ubench/abl/libpbx_oldgelu.so $T 300 python -u bench.py > gpurun_out/r3g_old_$i.json 2> gpurun_out/r3g_old_$i.err || exit 1
  python3 -c "import json;a=json.load(open('gpurun_out/r3g_new_$i.json'));b=json.load(open('gpurun_out/r3g_old_$i.json'));print('new',a['value'],a['ms_per_step'],'old',b['value'],b['ms_per_step'])"
done
