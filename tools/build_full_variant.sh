#!/bin/bash
# A whole libzp_hip.so built with extra flags from the lab sources (the
# product plus tools/patches/lab.patch; A/B of host + device code, e.g.
# tools/parse_one_latency.py --lib tools/variants/<name> with -DZP_ONE_STAMPS):
#   tools/build_full_variant.sh <name> [flags...]
cd "$(dirname "$0")/.." || exit 1
name=$1; shift
S=tools/variants/src_$name
rm -rf "$S" && mkdir -p "$S/zero-packet_amd" && cp -r zero-packet_amd/csrc "$S/zero-packet_amd/" \
  && cp -r include "$S/" && patch -s -p1 -d "$S" < tools/patches/lab.patch || exit 1
C=$S/zero-packet_amd/csrc
O=tools/variants/$name
mkdir -p "$O"
objs=()
for f in zp_parse zp_ctx zp_gen zp_fields zp_ring zp_build zp_stats; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC "$@" -c $C/$f.hip -o "$O/$f.o" || exit 1
  objs+=("$O/$f.o")
done
gcc -O3 -std=c11 -fPIC -c $C/zp_readers.c -o "$O/zp_readers.o" || exit 1
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$O/libzp_hip.so" "${objs[@]}" "$O/zp_readers.o" || exit 1
rm -f "$O"/*.o
