mkdir -p gpurun_out
timeout -k 10 500 python tools/kbench.py --variants g4,g16,wpe4 --configs c5,c3,c4 --rounds 5 > gpurun_out/r05ab_kb_g.log 2>&1 || exit $?
