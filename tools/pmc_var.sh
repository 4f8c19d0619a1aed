#!/bin/bash
# PMC passes per kernel variant: pmc_var.sh <config> <variant>... ("base" = in-tree lib).
# One counter group per rocprofv3 run, no tracing domains mixed in.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
cfg=$1; shift
for v in "$@"; do
  O=gpurun_out/pmc_$v
  mkdir -p $O
  if [ "$v" = base ]; then sel=""; else sel="--no-base --variants $v"; fi
  i=0
  for grp in "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" \
             "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
             "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD" \
             "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY"; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --pmc $grp -d $O/p$i -o p --output-format csv -- python3 tools/kbench.py --configs $cfg --rounds 1 --reps 3 $sel > $O/p$i.log 2>&1
    rc=$?
    echo "$v pass $i ($grp) rc=$rc"
    if [ $rc -ge 124 ]; then exit $rc; fi
  done
  python3 tools/pmc_summary.py $O > $O/summary.txt
  cat $O/summary.txt
done
