mkdir -p gpurun_out
timeout -k 10 60 tools/latency/lds_occ > gpurun_out/r05ae_lds_occ.log 2>&1 || exit $?
timeout -k 10 600 python tools/kbench.py --variants starts16,starts32 --configs c5,c3,c4,c6,c2 --rounds 6 > gpurun_out/r05ae_kb_starts.log 2>&1 || exit $?
