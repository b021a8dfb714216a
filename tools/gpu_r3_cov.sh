# Launcher coverage: the whole GPU suite with the coverage report written to gpurun_out/r3_cov
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3_cov
O=gpurun_out/r3_cov
PBX_LAUNCHER_REPORT=$O/launcher_coverage.txt timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
grep -E "general_global|rel-l2" $O/gpu_tests.log | tail -5 || true
cat $O/launcher_coverage.txt
