#!/bin/bash
# Another build of the engine library for same-box A/B runs (loaded through
# PSENGINE_LIB_AB):  bash tools/build_variant.sh <name> [-DSOME_DEFINE ...]
# -> go-libp2p-pubsub_amd/lib/libpsengine_<name>.so (git-ignored; travels)
set -euo pipefail
cd "$(dirname "$0")/.."
N=$1; shift
P=go-libp2p-pubsub_amd
O=$P/lib/obj_$N
mkdir -p $O
SRC="kernels.hip pull.hip flood.hip gbuild.hip graph.cpp plan.cpp run.cpp api.cpp tree.cpp dist.cpp codec.cpp pubsub.cpp"
for f in $SRC; do
  /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC -Wall -Iinclude -I$P/csrc "$@" -c $P/csrc/$f -o $O/$f.o &
done
for j in $(jobs -p); do wait $j || { echo "compile failed" >&2; rm -rf $O; exit 1; }; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -fPIC -shared $O/*.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib \
  -o $P/lib/libpsengine_$N.so
rm -rf $O $P/lib/libpsengine_$N.so.*
echo "built $P/lib/libpsengine_$N.so"
