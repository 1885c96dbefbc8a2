#!/bin/bash
# Build an A/B variant of the library: one source swapped (and/or extra -D flags), the other
# objects from build/obj.  tools/bin/libhnm_<tag>.so, loaded by setting HNM_LIB_PATH.
#   bash tools/build_variant.sh <tag> <source.hip> [hipcc flags...]
set -euo pipefail
TAG=$1; SRC=$2; shift 2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
python -c "import sys; sys.path.insert(0, '$ROOT'); from hnm_recommendation_amd.build import build_library; build_library(verbose=False)"
mkdir -p "$ROOT/tools/bin/obj_$TAG"
base=$(basename "$SRC" .hip)
# the variant source must carry the name of the object it replaces (e.g. an old version in
# another directory: git show HEAD:.../ncf_cert.hip > /tmp/old/ncf_cert.hip)
[ -f "$ROOT/build/obj/$base.o" ] || { echo "no build/obj/$base.o to replace"; exit 1; }
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I"$ROOT/hnm_recommendation_amd/csrc" -I"$ROOT/include" "$@" -c "$SRC" -o "$ROOT/tools/bin/obj_$TAG/$base.o"
objs=()
for o in "$ROOT"/build/obj/*.o; do
  [ "$(basename "$o" .o)" = "$base" ] && objs+=("$ROOT/tools/bin/obj_$TAG/$base.o") || objs+=("$o")
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$ROOT/tools/bin/libhnm_$TAG.so" "${objs[@]}" -L/opt/rocm/lib -lrccl
echo "built tools/bin/libhnm_$TAG.so"
