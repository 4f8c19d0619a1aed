mkdir -p gpurun_out
timeout -k 10 300 python tools/hdr_pattern.py --hdr 54,254 > gpurun_out/r05q_hdr_pattern.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05q_prof_c2 -o c2 -- python tools/kbench.py --c2cold --configs "" --rounds 5 > gpurun_out/r05q_c2cold.log 2>&1 || exit $?
