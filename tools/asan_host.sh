#!/bin/bash
# Host-side AddressSanitizer build of the C-ABI library and the driver in
# tests/asan/asan_driver.cpp ("-fsanitize=address host builds of the
# C-ABI shim").  The device code is compiled as usual; only the host half is instrumented
# (each -fsanitize= right after -Xarch_host).  No GPU needed: the driver exercises the
# entry points' validation and error paths.  Run from the repo root:  tools/asan_host.sh
set -euo pipefail
OUT=tools/bin/asan
mkdir -p "$OUT"
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
FLAGS=(--offload-arch=gfx950 -O1 -g -fPIC -std=c++17 -Wno-unused-result
       -Xarch_host -fsanitize=address -Xarch_host -fno-omit-frame-pointer)
objs=()
pids=()
rm -f "$OUT"/*.o        # never link a stale object left by an earlier run
for f in xtddft_amd/csrc/*.hip; do
  o="$OUT/$(basename "${f%.hip}").o"
  "$HIPCC" "${FLAGS[@]}" -c "$f" -o "$o" &
  pids+=($!)
  objs+=("$o")
done
for p in "${pids[@]}"; do wait "$p" || { echo "asan compile failed"; exit 1; }; done
echo 'const char* xt_build_id(void) { return "asan-host-build"; }' > "$OUT/xt_build_id.c"
gcc -O1 -fPIC -c "$OUT/xt_build_id.c" -o "$OUT/xt_build_id.o"
objs+=("$OUT/xt_build_id.o")
"$HIPCC" --offload-arch=gfx950 -shared -fPIC -fsanitize=address -o "$OUT/libxtddft_amd_asan.so" "${objs[@]}"
/opt/rocm/lib/llvm/bin/clang++ -O1 -g -fsanitize=address -fno-omit-frame-pointer tests/asan/asan_driver.cpp \
  -L"$OUT" -lxtddft_amd_asan -Wl,-rpath,"$(pwd)/$OUT" -o "$OUT/asan_driver"
ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 "$OUT/asan_driver"
