# Round-5 profiles: kernel-trace summaries (c3/c4/c5), PMC traffic (c3, c5),
# the fused/split choice, zp_parse_one latency, the bench line.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python tools/cols_policy.py --configs c3,c4,c5 > gpurun_out/r05l_cols_auto.log 2>&1 || exit $?
timeout -k 10 300 python tools/parse_one_latency.py --calls 5000 > gpurun_out/r05l_parse_one_latency.log 2>&1 || exit $?
bash tools/prof_config.sh c3 || exit $?
bash tools/prof_config.sh c4 || exit $?
bash tools/prof_config.sh c5 || exit $?
bash tools/pmc_traffic.sh r05 c3 || exit $?
bash tools/pmc_traffic.sh r05 c5 || exit $?
timeout -k 10 600 python bench.py > gpurun_out/r05l_bench.json 2> gpurun_out/r05l_bench.err || exit $?
