#!/bin/bash
# HBM traffic of the batched builder (tools/build_bench.py, 4M c3 frames):
# one PMC pass for the reads (FETCH_SIZE), one for the writes (WRITE_SIZE +
# TCC_EA0_WRREQ_sum), no tracing domains. Usage: tools/pmc_builder.sh <P>
# (payload bytes per frame, 0 = in-place chains). Summaries go to
# gpurun_out/pmc_build_P<P>/summary.txt.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
P=${1:-0}
O=gpurun_out/pmc_build_P$P
mkdir -p $O
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $O/rd -o p --output-format csv -- python3 tools/build_bench.py --reps 3 --payload $P --oracle-sample 0 > $O/rd.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE TCC_EA0_WRREQ_sum -d $O/wr -o p --output-format csv -- python3 tools/build_bench.py --reps 3 --payload $P --oracle-sample 0 > $O/wr.log 2>&1 || exit $?
{ grep "^build" $O/rd.log | head -1; python3 tools/pmc_summary.py $O/rd $O/wr; } > $O/summary.txt
cat $O/summary.txt
