#!/bin/bash
# rocprofv3 kernel-trace summary of bench.py on one config (no PMC, no other
# tracing domains): gpurun_out/prof_<cfg>/ holds the stats CSV and the bench
# line of the same run. Usage: tools/prof_config.sh <config> [extra bench args]
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
C=${1:-c3}; shift
O=gpurun_out/prof_$C
mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O -o run --output-format csv -- python3 bench.py --config $C --no-pcie --no-cpu --no-c5 "$@" > $O/bench.log 2>&1 || exit $?
grep '^{' $O/bench.log > $O/bench.json
f=$(find $O -name "*kernel_stats.csv" | head -1); cp "$f" $O/kernel_stats.csv
head -3 $O/kernel_stats.csv
