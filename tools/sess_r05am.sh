mkdir -p gpurun_out
timeout -k 10 700 python tools/kbench.py --variants aux2,aux0,aux18,aux3,aux17 --configs c5,c3,c4 --rounds 6 > gpurun_out/r05am_kb_aux.log 2>&1 || exit $?
