mkdir -p gpurun_out
timeout -k 10 600 python tools/kbench.py --variants notail,notail64 --configs c5,c3,c4,c6,c2 --rounds 6 > gpurun_out/r05ah_kb_notail.log 2>&1 || exit $?
