mkdir -p gpurun_out
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/r05d_smoke.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "parse_one or golden" > gpurun_out/r05d_tests_po.log 2>&1 || exit $?
timeout -k 10 200 python tools/parse_one_latency.py --calls 3000 --modes 5000 --threads 1 --lib tools/variants/stamps > gpurun_out/r05d_lat_stamps.log 2>&1 || exit $?
timeout -k 10 300 python tools/parse_one_latency.py --calls 3000 > gpurun_out/r05d_lat.log 2>&1 || exit $?
timeout -k 10 600 python tools/uc_ab.py --columns --arena-uc > gpurun_out/r05d_uc_ab.log 2>&1 || exit $?
timeout -k 10 200 python tools/hdr_pattern.py --uncached > gpurun_out/r05d_hdr_pattern_uc.log 2>&1 || exit $?
timeout -k 10 400 python bench.py > gpurun_out/r05d_bench.json 2> gpurun_out/r05d_bench.err || exit $?
timeout -k 10 300 python tools/build_bench.py --oracle-sample 200 --arena-mem uncached > gpurun_out/r05d_build_uc_P0.log 2>&1 || exit $?
timeout -k 10 300 python tools/build_bench.py --oracle-sample 200 --payload 200 > gpurun_out/r05d_build_P200.log 2>&1 || exit $?
timeout -k 10 300 python tools/build_bench.py --oracle-sample 200 --payload 200 --arena-mem uncached > gpurun_out/r05d_build_uc_P200.log 2>&1 || exit $?
timeout -k 10 200 python tools/parse_one_latency.py --calls 3000 --modes 5000 --threads 1 --lib tools/variants/ack16st > gpurun_out/r05d_lat_ack16st.log 2>&1 || exit $?
timeout -k 10 200 python tools/parse_one_latency.py --calls 3000 --modes 5000 --lib tools/variants/ack16 > gpurun_out/r05d_lat_ack16.log 2>&1 || exit $?
