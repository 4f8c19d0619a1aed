#!/bin/bash
# One GPU session: build check, GPU tests, smoke, bench, rocprof kernel trace.
# Every GPU step has its own time limit; a crash/abort/timeout (exit >= 124)
# ends the script immediately, ordinary test failures do not.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))" | tee -a $OUT/session.log
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a $OUT/session.log
  tail -5 "$OUT/$name.log" | tee -a $OUT/session.log
  if [ $rc -ge 124 ]; then echo "fatal rc=$rc in $name, stopping" | tee -a $OUT/session.log; exit $rc; fi
  return 0
}
i=0
for s in "$@"; do
  i=$((i+1))
  case $s in
    build)  step build 600 python __graft_entry__.py ;;
    tests)  step gpu_tests 1200 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    smoke)  step smoke 300 python __graft_entry__.py smoke ;;
    bench)  step bench 900 python bench.py ;;
    prof)   step prof 900 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --no-pcie ;;
    *) step "step$i" 900 bash -c "$s" ;;
  esac
done
