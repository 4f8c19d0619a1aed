#!/bin/bash
# HBM traffic of zp_parse_kernel under the bench workload (one PMC pass, no
# tracing domains). Writes profiles/<round>_traffic_<config>.json via
# tools/pmc_traffic.py. Usage: tools/pmc_traffic.sh [round] [config]
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
R=${1:-r01}; C=${2:-c3}
O=gpurun_out/traffic_$C
mkdir -p $O
timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum -d $O -o p --output-format csv -- python3 bench.py --config $C --steps 3 --warmup 1 --no-cpu --no-pcie --no-c5 > $O/bench.log 2>&1 || exit $?
python3 tools/pmc_traffic.py $O $C profiles/${R}_traffic_${C}.json && cp profiles/${R}_traffic_${C}.json gpurun_out/
