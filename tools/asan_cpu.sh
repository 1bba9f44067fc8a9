#!/bin/bash
# Host-side sanitizer builds on the CPU container (SURVEY §5 "ASan for host C ABI"; no GPU, no
# GPU sanitizer -- the pool has none):
#  1. libmpcblaster.so with the HOST side of every translation unit under AddressSanitizer and
#     UBSan (-Xarch_host, so device code is untouched), driven by tools/asan/capi_host.c through
#     every C-ABI entry point's validation and error paths (mpcb_create's no-device path included);
#  2. the plain-C oracle (oracle/c) under gcc's ASan + UBSan, run by tests/test_c_oracle.py
#     (MPCB_ORACLE_LIB points oracle/c_oracle.py at the instrumented build).
# Output under ${OUT:-/tmp/mpcb_asan}; exits non-zero on any sanitizer report or test failure.
set -euo pipefail
REPO=$(cd "$(dirname "$0")/.." && pwd)
OUT=${OUT:-/tmp/mpcb_asan}
cd "$REPO"
mkdir -p "$OUT"
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
SAN="-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=all -Xarch_host -fno-omit-frame-pointer"

echo "== 1. C ABI host side (hipcc, ASan + UBSan on the host code)"
python3 - "$OUT/libmpcblaster_asan.so" $SAN <<'PY'
import sys
sys.path.insert(0, sys.argv[0] and '.')
from mpc_blaster_amd import build as b
b.build(force=True, verbose=False, out=sys.argv[1], extra=sys.argv[2:] + ['-g'])
PY
$HIPCC -fsanitize=address,undefined -fno-sanitize-recover=all -g -x c "$REPO/tools/asan/capi_host.c" \
  -o "$OUT/capi_host" -L"$OUT" -l:libmpcblaster_asan.so -Wl,-rpath,"$OUT"
ASAN_OPTIONS=detect_leaks=1:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
  "$OUT/capi_host" > "$OUT/capi_host.log" 2>&1 || { cat "$OUT/capi_host.log"; exit 1; }
tail -1 "$OUT/capi_host.log"

echo "== 2. plain-C oracle (gcc, ASan + UBSan) under tests/test_c_oracle.py"
gcc -O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=all -march=x86-64-v3 \
  -fopenmp -fPIC -std=c99 -Wall -shared "$REPO/oracle/c/mpc_oracle.c" -o "$OUT/libmpc_oracle_asan.so" -lm
LD_PRELOAD="$(gcc -print-file-name=libasan.so):$(gcc -print-file-name=libubsan.so)" \
ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
MPCB_ORACLE_LIB="$OUT/libmpc_oracle_asan.so" \
  python3 -m pytest -q -p no:cacheprovider "$REPO/tests/test_c_oracle.py" > "$OUT/oracle_c.log" 2>&1 \
  || { tail -40 "$OUT/oracle_c.log"; exit 1; }
tail -1 "$OUT/oracle_c.log"
if grep -q "runtime error\|AddressSanitizer" "$OUT/oracle_c.log" "$OUT/capi_host.log"; then
  echo "sanitizer reports found"; exit 1
fi
echo asan_cpu_clean
