mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r05ai_gpu_tests.log 2>&1 || exit $?
timeout -k 10 600 python tools/kbench.py --variants tail --configs c5,c3,c4,c6 --rounds 8 > gpurun_out/r05ai_kb_tail.log 2>&1 || exit $?
