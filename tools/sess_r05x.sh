mkdir -p gpurun_out
timeout -k 10 400 python -u tools/fuzz_long.py 20 100000 > gpurun_out/r05x_fuzz_parse_long.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/fuzz_long.py 20 100000 0.85 > gpurun_out/r05x_fuzz_parse_long_repaired.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/fuzz_fast_ip.py 10 70000 > gpurun_out/r05x_fuzz_fast_ip.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/fuzz_columns_long.py 10 50000 > gpurun_out/r05x_fuzz_columns_long.log 2>&1 || exit $?
timeout -k 10 500 python -u tools/fuzz_builder_long.py 10 20000 > gpurun_out/r05x_fuzz_builder_long.log 2>&1 || exit $?
