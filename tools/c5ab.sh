cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 300 python bench.py > gpurun_out/c5ab_default_$i.log 2>&1 || exit $?
  timeout -k 10 300 python bench.py --no-pcie > gpurun_out/c5ab_nopcie_$i.log 2>&1 || exit $?
  timeout -k 10 300 python bench.py --no-cpu > gpurun_out/c5ab_nocpu_$i.log 2>&1 || exit $?
done
