bash tools/gpu_session.sh bench \
 "bash tools/pmc_traffic.sh r03v4 c3" \
 "bash tools/prof_config.sh c3" "bash tools/prof_config.sh c5" "bash tools/prof_config.sh c4" "bash tools/prof_config.sh c2 --steps 50" \
 "timeout -k 10 300 python tools/kbench.py --tiles --configs ''" \
 "timeout -k 10 300 python tools/fuzz_columns_long.py 6 60000" \
 "timeout -k 10 300 python tools/fuzz_long.py 6 60000 0.3"
