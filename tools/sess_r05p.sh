mkdir -p gpurun_out
timeout -k 10 300 python tools/hdr_pattern.py --hdr 54,108,254,1054 > gpurun_out/r05p_hdr_pattern.log 2>&1 || exit $?
timeout -k 10 300 python tools/build_bench.py --oracle-sample 200 > gpurun_out/r05p_build_P0.log 2>&1 || exit $?
timeout -k 10 300 python tools/build_bench.py --oracle-sample 200 --payload 200 > gpurun_out/r05p_build_P200.log 2>&1 || exit $?
timeout -k 10 300 python tools/build_bench.py --oracle-sample 200 --payload 1000 > gpurun_out/r05p_build_P1000.log 2>&1 || exit $?
timeout -k 10 400 python tools/kbench.py --configs c5,c3 --variants plainrec --rounds 6 > gpurun_out/r05p_kb_plainrec.log 2>&1 || exit $?
