mkdir -p gpurun_out
timeout -k 10 1500 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r05o_gpu_tests.log 2>&1 || exit $?
timeout -k 10 500 python tools/kbench.py --configs c5,c3,c4,c6,c2 --variants late,k2,norec --rounds 6 > gpurun_out/r05o_kb.log 2>&1 || exit $?
