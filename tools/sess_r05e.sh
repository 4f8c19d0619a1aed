mkdir -p gpurun_out
timeout -k 10 200 python tools/parse_one_latency.py --calls 2000 --modes 5000 --threads 1 --lib tools/variants/twice > gpurun_out/r05e_lat_twice.log 2>&1 || exit $?
timeout -k 10 200 python tools/parse_one_latency.py --calls 2000 --modes 5000 --threads 1 --lib tools/variants/ack16st > gpurun_out/r05e_lat_ack16st.log 2>&1 || exit $?
timeout -k 10 200 python tools/parse_one_latency.py --calls 3000 --modes 5000 --lib tools/variants/ack16 > gpurun_out/r05e_lat_ack16.log 2>&1 || exit $?
