#!/bin/bash
# Builds timing variants of the parse kernel into tools/variants/ (A/B only).
# The product sources carry no variant or ablation branches: the timing
# ablations (ZP_ABL_*, ZB_ABL_*), the diagnostic stamps (ZP_STAMPS,
# ZP_ONE_STAMPS, ZB_STAMPS, ZP_DBG_FBCOUNT) and the rejected layouts
# (ZP_NO_TAIL) come back from tools/patches/lab.patch, applied to a scratch
# copy of the sources under tools/variants/src.
cd "$(dirname "$0")/.." || exit 1
mkdir -p tools/variants
S=tools/variants/src
rm -rf "$S" && mkdir -p "$S/zero-packet_amd" && cp -r zero-packet_amd/csrc "$S/zero-packet_amd/" \
  && cp -r include "$S/" && patch -s -p1 -d "$S" < tools/patches/lab.patch || exit 1
C=$S/zero-packet_amd/csrc
build() {  # name flags...
  local name=$1; shift
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared "$@" \
     -o tools/variants/libzp_$name.so $C/zp_parse.hip $C/zp_parse_slots.hip || exit 1
}
buildb() {  # builder variants: name flags...
  local name=$1; shift
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared "$@" \
     -o tools/variants/libzb_$name.so $C/zp_build.hip $C/zp_parse.hip $C/zp_parse_slots.hip || exit 1
}
buildc() {  # column-view variants (parse + fields): name flags...
  local name=$1; shift
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared "$@" \
     -o tools/variants/libzc_$name.so $C/zp_fields.hip $C/zp_parse.hip $C/zp_parse_slots.hip || exit 1
}
for v in "$@"; do
  case $v in
    nostream)   build nostream -DZP_ABL_STREAM_OFF ;;
    fakewalk)   build fakewalk -DZP_ABL_FAKE_WALK ;;
    norec)      build norec -DZP_ABL_NOREC ;;
    norec_fakewalk) build norec_fakewalk -DZP_ABL_NOREC -DZP_ABL_FAKE_WALK ;;
    stamps)     build stamps -DZP_STAMPS ;;
    fbcount)    build fbcount -DZP_DBG_FBCOUNT ;;
    tailfree)   build tailfree -DZP_NO_TAIL=1 -DZP_STARTS=32 ;;
    b-*) name=${v%%:*}; flags=${v#*:}; buildb "${name#b-}" $flags ;;
    c-*) name=${v%%:*}; flags=${v#*:}; buildc "${name#c-}" $flags ;;
    *) name=${v%%:*}; flags=${v#*:}; build "$name" $flags ;;
  esac
done
