#!/bin/bash
# FETCH_SIZE / TCC_EA0_RDREQ by load width on a known byte count
# (tools/width_calib.py: 4 GiB read once per launch), one counter pass each.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/width
mkdir -p $O
timeout -k 10 120 python3 tools/width_calib.py > $O/plain.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o p --output-format csv -- python3 tools/width_calib.py > $O/fetch.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum -d $O/rdreq -o p --output-format csv -- python3 tools/width_calib.py > $O/rdreq.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE TCC_EA0_WRREQ_sum -d $O/wr -o p --output-format csv -- python3 tools/width_calib.py > $O/wr.log 2>&1 && timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_sum -d $O/dram -o p --output-format csv -- python3 tools/width_calib.py > $O/dram.log 2>&1
python3 tools/pmc_summary.py $O > $O/summary.txt 2>&1; cat $O/summary.txt
echo done
