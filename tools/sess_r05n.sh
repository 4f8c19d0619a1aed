mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "parse_one or golden or l4_far or jumbo" > gpurun_out/r05n_tests_po.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_l4_far.py tests/test_facade_cpp.py tests/test_debugfmt.py -m gpu > gpurun_out/r05n_tests_facades.log 2>&1 || exit $?
timeout -k 10 300 python tools/parse_one_latency.py --calls 5000 > gpurun_out/r05n_lat.log 2>&1 || exit $?
timeout -k 10 200 python tools/parse_one_latency.py --calls 3000 --modes 5000 --threads 1 --lib tools/variants/stamps > gpurun_out/r05n_lat_stamps.log 2>&1 || exit $?
timeout -k 10 200 python tools/parse_one_latency.py --calls 5000 --modes 5000 --lib tools/variants/batchtile > gpurun_out/r05n_lat_batchtile.log 2>&1 || exit $?
timeout -k 10 400 python tools/kbench.py --configs c5,c3,c4,c6 --variants earlyrec,norec --rounds 6 > gpurun_out/r05n_kb_earlyrec.log 2>&1 || exit $?
