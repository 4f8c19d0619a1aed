#!/bin/bash
# The batched builder's L2 read requests split into DRAM reads and the rest
# (TCC_EA0_RDREQ_sum vs TCC_EA0_RDREQ_DRAM_sum, one pass): re-reads of lines
# the same wave touched shortly before can be served by the Infinity Cache,
# which FETCH_SIZE counts too. Usage: tools/pmc_builder_dram.sh <P>...
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
for P in "$@"; do
  O=gpurun_out/pmc_build_dram_P$P
  mkdir -p $O
  timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum -d $O/rd -o p --output-format csv -- python3 tools/build_bench.py --reps 3 --payload $P --oracle-sample 0 > $O/rd.log 2>&1 || exit $?
  { grep "^build" $O/rd.log | head -1; python3 tools/pmc_summary.py $O/rd | grep -E "zp_build_fast_kernel|zp_parse_kernel"; } > $O/summary.txt
  cat $O/summary.txt
done
