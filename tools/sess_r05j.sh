mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "parse_one or golden" > gpurun_out/r05j_tests_po.log 2>&1 || exit $?
timeout -k 10 300 python tools/parse_one_latency.py --calls 5000 > gpurun_out/r05j_lat.log 2>&1 || exit $?
timeout -k 10 200 python tools/parse_one_latency.py --calls 3000 --modes 5000 --threads 1 --lib tools/variants/stamps > gpurun_out/r05j_lat_stamps.log 2>&1 || exit $?
timeout -k 10 300 python tools/kbench.py --configs c3,c5,c4 --variants r04 > gpurun_out/r05j_kb.log 2>&1 || exit $?
timeout -k 10 400 python tools/cols_policy.py --configs c3,c4,c5 > gpurun_out/r05j_cols_auto.log 2>&1 || exit $?
