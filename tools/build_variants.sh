#!/bin/bash
# Build libsmx variants with extra -D flags for A/B timing on the GPU box:
#   tools/build_variants.sh name1:"-DX=1 -DY=0" name2:"..."
# (environment knobs such as SMX_ABLATE / SMX_WIN_TGT need "-DSMX_DIAG=1")
# -> tools/_build/var_<name>/libsmx.so  (run with SMX_LIB=<that path>)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  out=$R/tools/_build/var_$name
  rm -rf "$out"; mkdir -p "$out"
  make -s -C "$R/semantic_merge_amd/csrc" OUT="$out/libsmx.so" BUILD="$out/obj" HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -Wno-unused-variable $flags" >/dev/null
  echo "built $name ($flags)"
done
