mkdir -p gpurun_out
timeout -k 10 200 python tools/parse_one_latency.py --calls 5000 --modes 5000 > gpurun_out/r05w_lat_base.log 2>&1 || exit $?
timeout -k 10 200 python tools/parse_one_latency.py --calls 5000 --modes 5000 --lib tools/variants/nopieces > gpurun_out/r05w_lat_nopieces.log 2>&1 || exit $?
timeout -k 10 200 python tools/parse_one_latency.py --calls 5000 --modes 5000 --threads 1 --lib tools/variants/stamps > gpurun_out/r05w_lat_stamps.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "parse_one" > gpurun_out/r05w_tests_one.log 2>&1 || exit $?
