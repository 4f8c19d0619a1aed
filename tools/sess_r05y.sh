mkdir -p gpurun_out
timeout -k 10 300 python tools/build_bench.py --oracle-sample 50 --payload 200 --variants fullsect --rounds 5 > gpurun_out/r05y_P200.log 2>&1 || exit $?
timeout -k 10 300 python tools/build_bench.py --oracle-sample 50 --payload 1000 --variants fullsect --rounds 5 > gpurun_out/r05y_P1000.log 2>&1 || exit $?
