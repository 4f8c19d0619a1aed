#!/bin/bash
# LDS pressure of zp_parse_kernel on one config (one PMC pass, no tracing).
# Usage: tools/pmc_lds.sh <config> [counters...]
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
C=${1:-c5}; shift
CTRS=${*:-SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES}
O=gpurun_out/pmc_lds_$C
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc $CTRS -d $O -o p --output-format csv -- python3 bench.py --config $C --steps 2 --warmup 1 --no-cpu --no-pcie > $O/bench.log 2>&1
