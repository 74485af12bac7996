set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
cp gladsgp_amd/libgpfit.so gpurun_out/.keep_lib.so
for v in pk_old pk_new; do
  cp _ab/libgpfit_$v.so gladsgp_amd/libgpfit.so
  echo "== $v"
  timeout -k 10 200 python tools/ab_packed.py > gpurun_out/r05d_ab_packed_$v.log 2>&1 || { cp gpurun_out/.keep_lib.so gladsgp_amd/libgpfit.so; exit 1; }
  cat gpurun_out/r05d_ab_packed_$v.log | grep points
done
cp gpurun_out/.keep_lib.so gladsgp_amd/libgpfit.so
