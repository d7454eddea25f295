#!/bin/bash
# Build a variant of the native library with extra HIP compile flags (A/B experiments):
#   tools/build_variant.sh NAME "-DLGBM_GATHER_ROWS=16"
# -> variants/NAME/lib_lightgbmv1_amd.so; run it with LIGHTGBM_AMD_LIB=variants/NAME/lib_lightgbmv1_amd.so
set -e
name=$1; extra=$2
rm -rf build_var/$name && mkdir -p build_var variants/$name
cp -a build build_var/$name
rm -f build_var/$name/device/*.hip.o
make -j8 BUILD=build_var/$name LIB=variants/$name/lib_lightgbmv1_amd.so HIPEXTRA="$extra" variants/$name/lib_lightgbmv1_amd.so > build_var/$name.log 2>&1
echo "built variants/$name ($extra)"
