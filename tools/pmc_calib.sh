#!/bin/bash
# FETCH_SIZE calibration on a known byte count (membw reads 13 GiB once per
# launch), then the parse kernel on c3 in the same session.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/calib
mkdir -p $O
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/membw -o p --output-format csv -- python3 tools/kbench.py --membw --configs c3 --rounds 1 --reps 2 > $O/membw.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_BUBBLE_sum -d $O/rdreq -o p --output-format csv -- python3 tools/kbench.py --membw --configs c3 --rounds 1 --reps 2 > $O/rdreq.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_32B_sum -d $O/dram -o p --output-format csv -- python3 tools/kbench.py --membw --configs c3 --rounds 1 --reps 2 > $O/dram.log 2>&1
echo done
