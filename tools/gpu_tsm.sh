# tsm block-size / occupancy variants on the tall-skinny probe (library copies swapped in)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
cp gladsgp_amd/libgpfit.so gpurun_out/.keep_tsm.so
: > gpurun_out/r05w_tsm.log
for rep in 1 2; do
  for v in 128_3 64_4 256_2; do
    cp _ab/libgpfit_tsm$v.so gladsgp_amd/libgpfit.so
    echo "== tsm $v" >> gpurun_out/r05w_tsm.log
    timeout -k 10 200 python tools/dbg/ts_probe.py 2>/dev/null | grep tsm >> gpurun_out/r05w_tsm.log || { cp gpurun_out/.keep_tsm.so gladsgp_amd/libgpfit.so; exit 1; }
  done
done
cp gpurun_out/.keep_tsm.so gladsgp_amd/libgpfit.so
cat gpurun_out/r05w_tsm.log
