mkdir -p gpurun_out
timeout -k 10 200 python tools/parse_one_latency.py --calls 2000 --modes 5000 --threads 1 --lib tools/variants/stamps > gpurun_out/r05f_lat_stamps.log 2>&1 || exit $?
timeout -k 10 400 python tools/cols_policy.py --configs c3,c4,c5 > gpurun_out/r05f_cols_auto.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_columns.py -m gpu > gpurun_out/r05f_tests_cols.log 2>&1 || exit $?
