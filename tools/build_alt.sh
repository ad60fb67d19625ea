#!/bin/bash
# Build an A/B variant of the default library: the named csrc files taken from git revision REV (or the
# working tree with REV=WORK) compiled with the extra flags in $EXTRA, every other object from this
# tree's build, linked into weatherconverter_amd/lib/${ALT:-alt}/libwc_kernels.so.
# Run it with WC_KERNEL_LIB=<that path> WC_ALLOW_STALE_LIB=1 (tools/ab_lib.sh, tools/wino_ab.py): the
# variant carries its own "alt:" digest, so the loader refuses it without that override.
# Usage: [ALT=name] [EXTRA="-DX=1"] [VARIANT=bf16] bash tools/build_alt.sh REV wc_conv6 [wc_igemm6 ...]
set -e
REV=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OBJ=$ROOT/weatherconverter_amd/lib/obj
OUT=$ROOT/weatherconverter_amd/lib/${ALT:-alt}
mkdir -p "$OUT"
python -c "import sys; sys.path.insert(0, '$ROOT'); from weatherconverter_amd import _build; _build.build()"
objs=""
for f in "$@"; do
  if [ "$REV" = "WORK" ]; then
    cp "$ROOT/weatherconverter_amd/csrc/$f.hip" "$ROOT/weatherconverter_amd/csrc/_alt_$f.hip"
  else
    git -C "$ROOT" show "$REV:weatherconverter_amd/csrc/$f.hip" > "$ROOT/weatherconverter_amd/csrc/_alt_$f.hip"
  fi
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics $EXTRA -I "$ROOT/include" \
    -Wno-unused-result -c "$ROOT/weatherconverter_amd/csrc/_alt_$f.hip" -o "$OUT/$f.o"
  rm "$ROOT/weatherconverter_amd/csrc/_alt_$f.hip"
  objs="$objs $OUT/$f.o"
done
# the variant's own digest ("alt:" + a hash of REV, EXTRA and the files): the loader refuses it unless
# WC_ALLOW_STALE_LIB=1, so an A/B or ablation build can never pass for the tree's library
ALTHASH="alt:$(echo "$REV $EXTRA $*" | sha256sum | cut -c1-16)"
printf 'extern "C" const char* wc_source_hash(void) { return "%s"; }\n' "$ALTHASH" > "$OUT/wc_srchash_alt.cpp"
/opt/rocm/bin/hipcc -x c++ -O2 -fPIC -c "$OUT/wc_srchash_alt.cpp" -o "$OUT/wc_srchash_alt.o"
excl="/($(echo "$@" | tr ' ' '|')|wc_srchash_bf16|wc_srchash_single16|wc_srchash_default)\.o$"
if [ -n "$VARIANT" ]; then
  # a single-piece build (VARIANT=bf16 / single16, EXTRA="-DWC_SINGLE16=2" / "=1"): its own objects where
  # the variant has them, the shared ones otherwise
  keep=$(ls "$OBJ/$VARIANT"/*.o | grep -v -E "$excl")
  for o in "$OBJ"/*.o; do
    [ -e "$OBJ/$VARIANT/$(basename "$o")" ] || keep="$keep $(echo "$o" | grep -v -E "$excl" || true)"
  done
else
  keep=$(ls "$OBJ"/*.o | grep -v -E "$excl")
fi
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$OUT/libwc_kernels.so" $keep $objs "$OUT/wc_srchash_alt.o"
echo "built $OUT/libwc_kernels.so ($REV $EXTRA: $*)"
