mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r05ar_gpu_tests.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05ar_smoke.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > gpurun_out/r05ar_bench.json 2> gpurun_out/r05ar_bench.err || exit $?
