#!/bin/bash
# Write traffic of the header write-back pattern (tools/hdr_pattern.py,
# per-lane whole-sector stores vs the whole wave on consecutive chunks) next
# to the in-place builder's (tools/build_bench.py): one PMC pass each,
# WRITE_SIZE + TCC_EA0_WRREQ_sum + TCC_EA0_WRREQ_64B_sum, no tracing.
# Usage: tools/pmc_writes.sh [hdr-bytes] [variant]. Summaries:
# gpurun_out/pmc_writes/summary.txt.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
H=${1:-54}
V=${2:-}
O=gpurun_out/pmc_writes${V:+_$V}
mkdir -p $O
C="WRITE_SIZE TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"
timeout -s KILL 120 rocprofv3 --pmc $C -d $O/hdr -o p --output-format csv -- python3 tools/hdr_pattern.py --hdr $H --policies ${POL:-0,4,5} --no-parse > $O/hdr.log 2>&1 || exit $?
X=""
[ -n "$V" ] && X="--variants $V"
timeout -s KILL 180 rocprofv3 --pmc $C -d $O/build -o p --output-format csv -- python3 tools/build_bench.py --reps 3 --oracle-sample 0 $X > $O/build.log 2>&1 || exit $?
{ cat $O/hdr.log; grep -E "^(write floor|build)" $O/build.log; python3 tools/pmc_summary.py $O/hdr $O/build; } > $O/summary.txt
cat $O/summary.txt
