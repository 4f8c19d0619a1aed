mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "parse_one" > gpurun_out/r05v_tests_one.log 2>&1 || exit $?
timeout -k 10 300 python tools/parse_one_latency.py --calls 5000 > gpurun_out/r05v_latency.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py > gpurun_out/r05v_tests.log 2>&1 || exit $?
