mkdir -p gpurun_out
timeout -k 10 1500 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r05m_gpu_tests.log 2>&1 || exit $?
timeout -k 10 400 python tools/kbench.py --configs c5,c3,c4 --variants mod,r04 --rounds 6 > gpurun_out/r05m_kb_fold.log 2>&1 || exit $?
timeout -k 10 400 python tools/kbench.py --configs c5,c3 --variants fakewalk,nol4hdr,nol1,nopseudo,norec > gpurun_out/r05m_kb_ablate.log 2>&1 || exit $?
