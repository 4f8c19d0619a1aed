mkdir -p gpurun_out
timeout -k 10 200 python tools/parse_one_latency.py --calls 3000 --modes 5000 --threads 1 --lib tools/variants/stamps > gpurun_out/r05c_lat_stamps.log 2>&1 || exit $?
timeout -k 10 300 python tools/cols_policy.py --configs c3,c4,c5 --lib cols96 > gpurun_out/r05c_cols96.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-c5 --no-cpu --no-pcie > gpurun_out/r05c_bench.json 2> gpurun_out/r05c_bench.err || exit $?
timeout -k 10 200 python tools/hdr_pattern.py > gpurun_out/r05c_hdr_pattern.log 2>&1 || exit $?
timeout -k 10 200 python tools/build_bench.py --oracle-sample 200 > gpurun_out/r05c_build_bench.log 2>&1 || exit $?
timeout -k 10 300 python tools/rec_pattern.py > gpurun_out/r05c_rec_pattern.log 2>&1 || exit $?
timeout -k 10 300 python tools/kbench.py --configs c5,c3,c4 --variants fold > gpurun_out/r05c_kb_fold.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "parse_one or golden" > gpurun_out/r05c_tests_po.log 2>&1 || exit $?
timeout -k 10 300 python tools/parse_one_latency.py --calls 3000 > gpurun_out/r05c_lat.log 2>&1 || exit $?
