mkdir -p gpurun_out
timeout -k 10 400 python tools/cols_policy.py --configs c3,c4,c5 > gpurun_out/r05k_cols_auto.log 2>&1 || exit $?
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/r05k_smoke.log 2>&1 || exit $?
timeout -k 10 1500 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r05k_gpu_tests.log 2>&1 || exit $?
