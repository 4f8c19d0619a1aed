mkdir -p gpurun_out
timeout -k 10 500 python tools/kbench.py --c2cold --variants pf2048,pf4096,pf4608,pf8192 --configs c3,c5 --rounds 5 > gpurun_out/r05aa_kb_pf.log 2>&1 || exit $?
