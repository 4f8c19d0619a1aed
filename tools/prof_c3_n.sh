#!/bin/bash
# rocprofv3 kernel-trace summaries of the c3 bench line in N separate
# processes (each with its own arena allocation, so its own placement):
# gpurun_out/prof_c3_<k>/ for k = 1..N.   Usage: tools/prof_c3_n.sh [N]
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
N=${1:-4}
for k in $(seq 1 $N); do
  O=gpurun_out/prof_c3_$k
  mkdir -p $O
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O -o run --output-format csv -- python3 bench.py --config c3 --no-pcie --no-cpu --no-c5 --steps 20 --warmup 5 > $O/bench.log 2>&1 || exit $?
  grep '^{' $O/bench.log > $O/bench.json
  f=$(find $O -name "*kernel_stats.csv" | head -1); cp "$f" $O/kernel_stats.csv
done
