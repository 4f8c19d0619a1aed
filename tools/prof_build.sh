#!/bin/bash
# rocprofv3 kernel-trace summaries of the batched builder (tools/build_bench.py,
# 4M c3 frames, in place and with 200 / 1000-B payloads from per-frame blob
# ranges), then its PMC write/read pass at P = 1000 (tools/pmc_builder.sh).
# Outputs under gpurun_out/prof_build_P<P>/ and gpurun_out/pmc_build_P1000/.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
for P in 0 200 1000; do
  O=gpurun_out/prof_build_P$P; mkdir -p $O
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O -o run --output-format csv -- python3 tools/build_bench.py --payload $P --oracle-sample 0 --reps 10 > $O/bench.log 2>&1 || exit $?
  f=$(find $O -name "*kernel_stats.csv" | head -1); cp "$f" $O/kernel_stats.csv
done
bash tools/pmc_builder.sh 1000
