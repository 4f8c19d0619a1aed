#!/bin/bash
# HBM traffic of the batched builder (tools/build_bench.py, 4M c3 frames):
# one PMC pass for the reads (FETCH_SIZE), one for the writes (WRITE_SIZE +
# TCC_EA0_WRREQ_sum), no tracing domains. Usage: tools/pmc_builder.sh <P> [variant]
# (payload bytes per frame, 0 = in-place chains; a tools/variants/libzb_<variant>.so
# build instead of the library, whose output may differ: probes). Summaries go to
# gpurun_out/pmc_build_P<P>[_<variant>]/summary.txt.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
P=${1:-0}
V=${2:-}
O=gpurun_out/pmc_build_P$P${V:+_$V}
X=""
[ -n "$V" ] && X="--variants $V --no-base"
mkdir -p $O
run() {  # run <dir> <counters...>: a probe variant may fail its round trip (rc 1)
  local d=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" -d $O/$d -o p --output-format csv -- python3 tools/build_bench.py --reps 3 --payload $P --oracle-sample 0 $X > $O/$d.log 2>&1
  local rc=$?
  if [ $rc -ne 0 ] && { [ -z "$V" ] || [ $rc -ge 124 ]; }; then exit $rc; fi
  return 0
}
run rd FETCH_SIZE
run wr WRITE_SIZE TCC_EA0_WRREQ_sum
{ grep "^build" $O/rd.log | head -1; python3 tools/pmc_summary.py $O/rd $O/wr; } > $O/summary.txt
cat $O/summary.txt
