#!/bin/bash
# ASan + UBSan build of liblsp_hip.so's host code (every source; the device
# code is unchanged: each -fsanitize= sits behind -Xarch_host) and of the fuzz
# driver (driver.cpp), then a run over a proof and the CBOR fixtures.
#
#   tools/sanitize/run.sh <proof.bin> [iterations] [seed]
#
# Objects and binaries go to tools/sanitize/_build (git-ignored); sources are
# rebuilt only when newer than their object.  CPU only: no GPU is used.
set -eo pipefail
HERE=$(cd "$(dirname "$0")" && pwd)
ROOT=$(cd "$HERE/../.." && pwd)
CSRC=$ROOT/linea_stark_prover_amd/csrc
OUT=$HERE/_build
mkdir -p "$OUT"
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
SAN="-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=undefined -Xarch_host -fno-omit-frame-pointer"
FLAGS="-O1 -g -std=c++17 -fPIC --offload-arch=gfx950 -Xarch_host -mbmi2 -Xarch_host -madx -I $ROOT/include $SAN"
SRCS=$(python3 -c "import sys; sys.path.insert(0, '$ROOT'); from linea_stark_prover_amd.build import SOURCES; print(' '.join(SOURCES))")
newest_hdr=$(ls -t "$CSRC"/*.hpp "$CSRC"/*.inc "$ROOT/include/lsp.h" | head -1)
pids=()
for s in $SRCS; do
  o=$OUT/${s%.*}.o
  if [ ! -f "$o" ] || [ "$CSRC/$s" -nt "$o" ] || [ "$newest_hdr" -nt "$o" ]; then
    x=""; case $s in *.cpp) x="-x hip";; esac
    $HIPCC $FLAGS $x -c "$CSRC/$s" -o "$o" &
    pids+=($!)
    if [ ${#pids[@]} -ge 8 ]; then wait "${pids[0]}"; pids=("${pids[@]:1}"); fi
  fi
done
for p in "${pids[@]}"; do wait "$p"; done
objs=$(for s in $SRCS; do echo -n "$OUT/${s%.*}.o "; done)
$HIPCC -shared --offload-arch=gfx950 -fno-gpu-sanitize -fsanitize=address,undefined -shared-libsan -o "$OUT/liblsp_hip_asan.so" $objs -lpthread -ldl
# the driver is plain host C++ against include/lsp.h, built by the same clang
CLANG=/opt/rocm/lib/llvm/bin/clang++
RTDIR=$(dirname "$($CLANG -print-file-name=libclang_rt.asan-x86_64.so)")
[ -f "$RTDIR/libclang_rt.asan-x86_64.so" ] || RTDIR=$(dirname "$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)")
$CLANG -O1 -g -std=c++17 -fsanitize=address,undefined -shared-libsan -fno-omit-frame-pointer -I "$ROOT/include" \
  "$HERE/driver.cpp" -o "$OUT/driver" -L "$OUT" -llsp_hip_asan -Wl,-rpath,"$OUT" -Wl,-rpath,"$RTDIR"
# leak checking is off: the HIP runtime's own one-time allocations are not ours
ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
  "$OUT/driver" "${3:-1}" "${2:-300}" "$1" "$ROOT/tests/golden/perm_small.cbor" "$ROOT/tests/golden/lookup_small.cbor"
