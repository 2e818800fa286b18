#!/bin/bash
# build/var/NAME/libmhe.so: an A/B variant of libmhe.so with extra compile flags, e.g.
#   bash scripts/build_var.sh base -DMHE_ROW_PRE=0
# Loaded by the Python binding with MHE_LIB_PATH=build/var/NAME/libmhe.so.
set -eu
NAME=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
D=$ROOT/build/${VARDIR:-var}/$NAME
mkdir -p "$D"
make -s -C "$ROOT/fhe-gpt-2_amd/csrc" OUT="$D/libmhe.so" BUILD="$D/obj" \
  HIPFLAGS="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -fvisibility=hidden -ffp-contract=off -Wall -Wno-unused-function $*"
