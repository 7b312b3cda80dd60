#!/bin/bash
# Build compile-time variants of libplssvm_mi355x.so into variants/<name>.so (A/B on the box with
# PLSSVM_MI_LIB=variants/<name>.so). usage: tools/variants.sh name "EXTRA flags" [name "flags"]...
set -e
root=$(cd "$(dirname "$0")/.." && pwd)
while [ $# -ge 2 ]; do
  make -s -C "$root/plssvm_sparse_fp22_amd/csrc" -j8 OUT="$root/variants/$1.so" BUILD="$root/build/var_$1" EXTRA="$2"
  shift 2
done
