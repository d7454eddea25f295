#!/bin/bash
# Golden oracle: the reference's CPU command line program built from
# its sources in a scratch copy (USE_GPU=OFF), for tests/test_golden.py.  Nothing prebuilt from
# the reference is used.  usage: tools/build_golden.sh [OUT_DIR=/tmp/refbuild]
set -e
REF=${REF:-/root/reference}
OUT=${1:-/tmp/refbuild}
if [ -x "$OUT/lightgbm" ]; then echo "$OUT/lightgbm"; exit 0; fi
rm -rf "$OUT" && mkdir -p "$OUT"
cp -r "$REF/CMakeLists.txt" "$REF/src" "$REF/include" "$OUT/"
chmod -R u+w "$OUT"
cmake -S "$OUT" -B "$OUT/build" -DUSE_GPU=OFF -DCMAKE_POLICY_VERSION_MINIMUM=3.5 -DCMAKE_BUILD_TYPE=Release > "$OUT/cmake.log" 2>&1
make -C "$OUT/build" -j"${JOBS:-6}" lightgbm > "$OUT/make.log" 2>&1
echo "$OUT/lightgbm"
