#!/bin/bash
# Build weatherconverter_amd/lib/alt/libwc_kernels.so for a same-box A/B (tools/gpu_ab_lib.sh,
# tools/gpu_probe.sh): the named csrc files taken from git revision REV, every other object from
# this tree's build.  Usage: bash tools/build_alt.sh REV wc_conv6 [wc_igemm6 ...]
set -e
REV=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OBJ=$ROOT/weatherconverter_amd/lib/obj
ALT=$ROOT/weatherconverter_amd/lib/alt
mkdir -p "$ALT"
python -c "import sys; sys.path.insert(0, '$ROOT'); from weatherconverter_amd import _build; _build.build()"
objs=""
for f in "$@"; do
  git -C "$ROOT" show "$REV:weatherconverter_amd/csrc/$f.hip" > "$ROOT/weatherconverter_amd/csrc/_alt_$f.hip"
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -I "$ROOT/include" \
    -Wno-unused-result -c "$ROOT/weatherconverter_amd/csrc/_alt_$f.hip" -o "$ALT/$f.o"
  rm "$ROOT/weatherconverter_amd/csrc/_alt_$f.hip"
  objs="$objs $ALT/$f.o"
done
keep=$(ls "$OBJ"/*.o | grep -v -E "/($(echo "$@" | tr ' ' '|'))\.o$")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$ALT/libwc_kernels.so" $keep $objs
echo "built $ALT/libwc_kernels.so ($REV: $*)"
