# Build and run the diagonal-factor micro-benchmark for leaf variants (LEAF_MASKED=0/1)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for v in ${LEAF_VARIANTS:-0 1}; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-mfma-vgpr-form -Xclang -target-feature -Xclang +enable-ds128 -DLEAF_MASKED=$v tools/dbg/diag_micro.hip -o /tmp/diag_micro_m$v > /dev/null 2>&1 || exit 1
done
for rep in 1 2; do
  for v in ${LEAF_VARIANTS:-0 1}; do
    echo "== LEAF_MASKED=$v" >> gpurun_out/leaf_masked.log
    timeout -k 10 60 /tmp/diag_micro_m$v >> gpurun_out/leaf_masked.log 2>&1 || exit 1
  done
done
grep -E "==|rep 3|max\|" gpurun_out/leaf_masked.log
