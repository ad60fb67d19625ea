#!/bin/bash
# Host-side AddressSanitizer build of the whole C ABI (every csrc/*.hip), linked into
# abi_validation.cpp and run on the CPU (no GPU needed; GPU ASan is not available on this pool).
# Usage: bash tools/asan/run.sh   (from the repo root; ~3 min, 8 parallel compiles)
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
OUT=$ROOT/tools/asan/_build
mkdir -p "$OUT"
FLAGS="-O1 -g -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -I $ROOT/include -Wno-unused-result"
ASAN="-Xarch_host -fsanitize=address -Xarch_host -fno-omit-frame-pointer"
ls "$ROOT"/weatherconverter_amd/csrc/*.hip | xargs -P 8 -I{} sh -c \
  "/opt/rocm/bin/hipcc $FLAGS $ASAN -c {} -o $OUT/\$(basename {} .hip).o"
/opt/rocm/bin/hipcc $FLAGS $ASAN -c "$ROOT/tools/asan/abi_validation.cpp" -o "$OUT/abi_validation.o"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -fsanitize=address "$OUT"/*.o -o "$OUT/abi_validation"
ASAN_OPTIONS=detect_leaks=1:abort_on_error=0 "$OUT/abi_validation"
