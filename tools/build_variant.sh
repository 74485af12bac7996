#!/bin/bash
# Link a variant of libgpfit with one source file replaced (A/B builds for tools/ab_libs.py and
# tools/ab_bench_libs.sh):
#   tools/build_variant.sh path/to/variant.hip out.so [replaced object: chol | predict | gram ...]
# The other objects come from gladsgp_amd/_obj (the current build).
set -e
cd "$(dirname "$0")/.."
SRC=$1; OUT=$2; REP=${3:-chol}
OBJ=$(mktemp --suffix=.o)
cp "$SRC" gladsgp_amd/csrc/.variant.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-function \
  -mllvm -amdgpu-mfma-vgpr-form -Xclang -target-feature -Xclang +enable-ds128 \
  -c gladsgp_amd/csrc/.variant.hip -o "$OBJ" 2>&1 | grep -v ds128 || true
rm -f gladsgp_amd/csrc/.variant.hip
objs=""
for f in gram chol predict linalg profile blas eig comm rng mcmc host_rng field; do
  [ "$f" = "$REP" ] || objs="$objs gladsgp_amd/_obj/$f.o"
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT" "$OBJ" $objs -ldl
rm -f "$OBJ"
echo "$OUT"
