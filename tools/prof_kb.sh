#!/bin/bash
# rocprofv3 kernel-trace summary of a tools/kbench.py run (per-kernel averages
# of A/B builds): tools/prof_kb.sh <out-name> <kbench args...>
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/profkb_$1; shift
mkdir -p $O
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O -o run --output-format csv -- python3 tools/kbench.py "$@" > $O/kbench.log 2>&1 || exit $?
f=$(find $O -name "*kernel_stats.csv" | head -1); cp "$f" $O/kernel_stats.csv
cat $O/kbench.log; cut -d, -f1-4 $O/kernel_stats.csv | grep -E "zp_|Name"
