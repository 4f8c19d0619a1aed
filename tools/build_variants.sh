#!/bin/bash
# Builds timing variants of the parse kernel into tools/variants/ (A/B only).
cd "$(dirname "$0")/.." || exit 1
mkdir -p tools/variants
C=zero-packet_amd/csrc
build() {  # name flags...
  local name=$1; shift
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared "$@" \
     -o tools/variants/libzp_$name.so $C/zp_parse.hip || exit 1
}
buildb() {  # builder variants: name flags...
  local name=$1; shift
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared "$@" \
     -o tools/variants/libzb_$name.so $C/zp_build.hip $C/zp_parse.hip || exit 1
}
buildc() {  # column-view variants (parse + fields): name flags...
  local name=$1; shift
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared "$@" \
     -o tools/variants/libzc_$name.so $C/zp_fields.hip $C/zp_parse.hip || exit 1
}
for v in "$@"; do
  case $v in
    nostream)   build nostream -DZP_ABL_STREAM_OFF ;;
    fakewalk)   build fakewalk -DZP_ABL_FAKE_WALK ;;
    streamonly) build streamonly -DZP_ABL_FAKE_WALK -DZP_ABL_WIN_OFF ;;
    unroll8)    build unroll8 -DZP_UNROLL=8 ;;
    unroll2)    build unroll2 -DZP_UNROLL=2 ;;
    b-*) name=${v%%:*}; flags=${v#*:}; buildb "${name#b-}" $flags ;;
    c-*) name=${v%%:*}; flags=${v#*:}; buildc "${name#c-}" $flags ;;
    *) name=${v%%:*}; flags=${v#*:}; build "$name" $flags ;;
  esac
done
