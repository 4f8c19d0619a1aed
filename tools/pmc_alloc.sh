#!/bin/bash
# UTCL1 translation counters of zp_parse_kernel over the placements of
# tools/alloc_probe.py (one process, several arena placements), one PMC pass.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/pmc_alloc
mkdir -p $O
timeout -s KILL 240 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE -d $O -o p --output-format csv -- python3 tools/alloc_probe.py --steps 3 --copies 6 --parse-only > $O/probe.log 2>&1
