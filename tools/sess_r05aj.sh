mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r05aj_gpu_tests.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05aj_smoke.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > gpurun_out/r05aj_bench.json 2> gpurun_out/r05aj_bench.err || exit $?
timeout -k 10 300 python tools/parse_one_latency.py --calls 5000 > gpurun_out/r05aj_latency.log 2>&1 || exit $?
