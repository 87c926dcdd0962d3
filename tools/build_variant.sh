#!/bin/bash
# Build a variant of librrt with extra compile flags into ab_var/librrt_NAME.so without
# touching the in-tree build (A/B runs load it through RRT_LIB).
# Usage: tools/build_variant.sh NAME "-DRRT_TAIL_PRIO=0 ..."
set -e
cd "$(dirname "$0")/.."
NAME=$1; FLAGS=$2
T=$(mktemp -d)
mkdir -p "$T/pkg" ab_var
cp -r relativistic-ray-tracer_amd/csrc relativistic-ray-tracer_amd/Makefile "$T/pkg/"
cp -r include "$T/include"
make -C "$T/pkg" -j8 EXTRA="$FLAGS" librrt.so > /dev/null
cp "$T/pkg/librrt.so" "ab_var/librrt_$NAME.so"
rm -rf "$T"
echo "ab_var/librrt_$NAME.so"
