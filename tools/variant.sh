#!/bin/bash
# Build an A/B variant of libplacement.so from a copy of the current csrc (optionally with extra
# compiler flags) into build_variants/<name>.so; load it with PE_LIBRARY=$PWD/build_variants/<name>.so.
#   tools/variant.sh <name> [EXTRA flags...]      e.g. tools/variant.sh wprof -DPE_WALK_PROF
#   (VARIANT_DIR=<dir>: build there instead, e.g. rb/ so that it travels with gpurun)
set -e
name=$1; shift
root=$(cd "$(dirname "$0")/.." && pwd)
src=$root/training-operator_amd/.v_$name     # same depth as csrc: the Makefile's ../../include holds
rm -rf "$src"
vdir=${VARIANT_DIR:-$root/build_variants}; mkdir -p "$vdir"
cp -r "$root/training-operator_amd/csrc" "$src"
rm -rf "$src/build"
make -s -j8 -C "$src" ARCH=gfx950 OUT="$vdir/$name.so" EXTRA="$*" 2>&1 | grep -v "Winline-asm\|clobber\|^ *[0-9]* |\|^ *|\|note:" || true
rm -rf "$src"
ls -la "$vdir/$name.so"
