mkdir -p gpurun_out
timeout -k 10 200 python tools/parse_one_latency.py --calls 5000 --modes 5000 > gpurun_out/r05ak_lat_base.log 2>&1 || exit $?
timeout -k 10 200 python tools/parse_one_latency.py --calls 5000 --modes 5000 --lib tools/variants/poll2 > gpurun_out/r05ak_lat_poll2.log 2>&1 || exit $?
timeout -k 10 200 python tools/parse_one_latency.py --calls 5000 --modes 5000 > gpurun_out/r05ak_lat_base2.log 2>&1 || exit $?
timeout -k 10 200 python tools/parse_one_latency.py --calls 5000 --modes 5000 --lib tools/variants/poll2 > gpurun_out/r05ak_lat_poll2b.log 2>&1 || exit $?
