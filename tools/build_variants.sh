#!/bin/bash
# Build several chol.hip variants in parallel into _ab/libgpfit_<name>.so (A/B for
# tools/ab_libs.py); the other objects come from gladsgp_amd/_obj (the current build).
#   tools/build_variants.sh name1:path1.hip name2:path2.hip ...
set -e
cd "$(dirname "$0")/.."
mkdir -p _ab
objs=""
for f in gram predict linalg profile blas eig comm rng mcmc host_rng; do objs="$objs gladsgp_amd/_obj/$f.o"; done
pids=""
for spec in "$@"; do
  name=${spec%%:*}; src=${spec#*:}
  (cp "$src" gladsgp_amd/csrc/.var_$name.hip &&
   /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-function \
     -mllvm -amdgpu-mfma-vgpr-form -Xclang -target-feature -Xclang +enable-ds128 \
     -c gladsgp_amd/csrc/.var_$name.hip -o _ab/chol_$name.o 2>&1 | { grep -v ds128 || true; };
   rm -f gladsgp_amd/csrc/.var_$name.hip;
   /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o _ab/libgpfit_$name.so \
     _ab/chol_$name.o $objs -ldl && echo "_ab/libgpfit_$name.so") &
  pids="$pids $!"
done
for p in $pids; do wait $p; done
