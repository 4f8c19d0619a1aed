mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "parse_one or golden" > gpurun_out/r05g_tests_po.log 2>&1 || exit $?
timeout -k 10 200 python tools/parse_one_latency.py --calls 3000 --modes 5000 --threads 1 --lib tools/variants/stamps > gpurun_out/r05g_lat_stamps.log 2>&1 || exit $?
timeout -k 10 300 python tools/parse_one_latency.py --calls 5000 > gpurun_out/r05g_lat.log 2>&1 || exit $?
timeout -k 10 200 python tools/parse_one_latency.py --calls 3000 --modes 5000 --threads 1 --lib tools/variants/ack16st > gpurun_out/r05g_lat_ack16st.log 2>&1 || exit $?
timeout -k 10 300 python tools/parse_one_latency.py --calls 5000 --modes 5000 --lib tools/variants/ack16 > gpurun_out/r05g_lat_ack16.log 2>&1 || exit $?
timeout -k 10 400 python tools/cols_policy.py --configs c3,c4,c5 > gpurun_out/r05g_cols_auto.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_columns.py -m gpu > gpurun_out/r05g_tests_cols.log 2>&1 || exit $?
