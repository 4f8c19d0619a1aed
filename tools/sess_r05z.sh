mkdir -p gpurun_out
bash tools/prof_config.sh c3 || exit $?
bash tools/prof_config.sh c4 || exit $?
bash tools/prof_config.sh c5 || exit $?
bash tools/pmc_traffic.sh r05 c4 || exit $?
