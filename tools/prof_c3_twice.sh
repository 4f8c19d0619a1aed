#!/bin/bash
# Two rocprofv3 kernel-trace summaries of the c3 bench line in two processes
# (each with its own arena allocation): gpurun_out/prof_c3_a, prof_c3_b.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
for k in a b; do
  O=gpurun_out/prof_c3_$k
  mkdir -p $O
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O -o run --output-format csv -- python3 bench.py --config c3 --no-pcie --no-cpu --no-c5 > $O/bench.log 2>&1 || exit $?
  grep '^{' $O/bench.log > $O/bench.json
  f=$(find $O -name "*kernel_stats.csv" | head -1); cp "$f" $O/kernel_stats.csv
done
