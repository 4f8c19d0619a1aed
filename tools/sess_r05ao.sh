mkdir -p gpurun_out
timeout -k 10 300 python tools/fbcount.py fbc,fbclru2 > gpurun_out/r05ao_fbcount.log 2>&1 || exit $?
timeout -k 10 600 python tools/kbench.py --variants lru2 --configs c4,c5,c3,c6 --rounds 6 > gpurun_out/r05ao_kb_lru2.log 2>&1 || exit $?
