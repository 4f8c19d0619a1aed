mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "min_size or config2 or config1 or small_batches or layouts" > gpurun_out/r05r_tests.log 2>&1 || exit $?
timeout -k 10 400 python tools/kbench.py --c2cold --variants notiny2 --configs c3,c5,c1 --rounds 5 > gpurun_out/r05r_kb_tiny2.log 2>&1 || exit $?
