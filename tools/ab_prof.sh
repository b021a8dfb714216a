# Per-kernel A/B: rocprofv3 kernel stats of the bench step with the in-tree library and with
# tools/ubench/abl/libpbx_<name>.so.   usage: bash tools/ab_prof.sh <name> [bench args]   (then tools/ab_profcmp.py)
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
name=$1; shift
rm -rf $R/gpurun_out/abp_new $R/gpurun_out/abp_$name
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/abp_new -- python3 $R/bench.py --steps 5 --warmup 3 "$@" > $R/gpurun_out/abp_new.log 2>&1 || exit 1
PBX_HIP_LIB=$R/tools/ubench/abl/libpbx_$name.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/abp_$name -- python3 $R/bench.py --steps 5 --warmup 3 "$@" > $R/gpurun_out/abp_$name.log 2>&1 || exit 1
