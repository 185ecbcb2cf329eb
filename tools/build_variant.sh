#!/bin/bash
# Builds an experiment variant of librt_amd.so into cpu-raytracing-rt_amd/build_<name>/
# with extra compiler flags (e.g. -DRT_ONLY_C2 -DSOME_SWITCH).  Product build: make.
#   bash tools/build_variant.sh <name> [flags...]
set -e
cd "$(dirname "$0")/../cpu-raytracing-rt_amd/csrc"
NAME=$1; shift
make -s -j4 OUT=../build_$NAME EXTRA="$*" > /dev/null
echo "built cpu-raytracing-rt_amd/build_$NAME/librt_amd.so ($*)"
