#!/bin/bash
# Build the kernel library from a git revision's csrc/ into tools/ubench/abl/libpbx_<name>.so
# (A/B runs: PBX_HIP_LIB=tools/ubench/abl/libpbx_<name>.so python bench.py ...).
# usage: tools/build_variant.sh <git-rev> <name>
set -e
rev=$1; name=$2
d=$(mktemp -d)
git archive "$rev" proteinbert_pytorch_replication_amd/ops/csrc | tar -x -C "$d"
src=$d/proteinbert_pytorch_replication_amd/ops/csrc
mkdir -p tools/ubench/abl
objs=""
for f in "$src"/*.hip; do
  o="$d/$(basename "$f" .hip).o"
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -ffp-contract=fast -fno-slp-vectorize -Wno-unused-result -I "$src" -c "$f" -o "$o" &
  objs="$objs $o"
done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o tools/ubench/abl/libpbx_$name.so $objs
rm -rf "$d"
echo tools/ubench/abl/libpbx_$name.so
