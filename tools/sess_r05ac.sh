mkdir -p gpurun_out
timeout -k 10 500 python tools/kbench.py --variants fakewalk,norec,fwnr --configs c5,c3 --tiles --rounds 5 > gpurun_out/r05ac_kb_abl.log 2>&1 || exit $?
