#!/bin/bash
# The CPU suite with the host-side C code (oracle, host generator) built
# under AddressSanitizer + UBSan; restores the normal builds afterwards.
cd "$(dirname "$0")/.." || exit 1
set -e
F="-O1 -g -std=c11 -fsanitize=address,undefined -fno-omit-frame-pointer -fPIC -shared"
gcc $F -o oracle/libzp_oracle.so oracle/zp_oracle.c -lpthread
gcc $F -o zero-packet_amd/libzp_host.so zero-packet_amd/csrc/zp_host.c -lpthread
set +e
ASAN_OPTIONS=detect_leaks=0:halt_on_error=1 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
LD_PRELOAD="$(gcc -print-file-name=libasan.so) $(gcc -print-file-name=libubsan.so)" \
  python -m pytest tests -q -m "not gpu" -p no:cacheprovider
rc=$?
make -s -C oracle -B
gcc -O2 -std=c11 -Wall -Wextra -fPIC -shared -o zero-packet_amd/libzp_host.so zero-packet_amd/csrc/zp_host.c -lpthread
exit $rc
