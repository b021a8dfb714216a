#!/bin/bash
# Build the kernel library from the WORKING TREE's csrc/ (or SRC=<dir>, e.g. an older checkout for a same-box
# A/B) with extra compile flags into tools/ubench/abl/libpbx_<name>.so (PBX_HIP_LIB=... python tools/...).
# usage: tools/ubench/build_flags.sh <name> [hipcc flags...]
set -e
name=$1; shift
src=${SRC:-proteinbert_pytorch_replication_amd/ops/csrc}
d=$(mktemp -d)
mkdir -p tools/ubench/abl
objs=""
for f in "$src"/*.hip; do
  o="$d/$(basename "$f" .hip).o"
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -ffp-contract=fast-honor-pragmas -fno-slp-vectorize -Wno-unused-result -I "$src" "$@" -c "$f" -o "$o" &
  objs="$objs $o"
done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o tools/ubench/abl/libpbx_$name.so $objs
rm -rf "$d"
echo tools/ubench/abl/libpbx_$name.so
