mkdir -p gpurun_out
timeout -k 10 400 python tools/kbench.py --c2cold --variants notiny2,t2nocold,t2s1nocold,t2s64nocold --configs c5 --rounds 5 > gpurun_out/r05s_kb_tiny2.log 2>&1 || exit $?
