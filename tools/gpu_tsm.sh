# Tall-skinny variants on the tall-skinny probe (library copies swapped in)
#   TS_LIBS="_ab/a.so _ab/b.so" bash tools/gpu_tsm.sh   -> gpurun_out/r05w_ts.log
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
cp gladsgp_amd/libgpfit.so gpurun_out/.keep_tsm.so
: > gpurun_out/r05w_ts.log
for rep in 1 2; do
  for lib in $TS_LIBS; do
    cp $lib gladsgp_amd/libgpfit.so
    echo "== $(basename $lib)" >> gpurun_out/r05w_ts.log
    timeout -k 10 200 python tools/dbg/ts_probe.py 2>/dev/null | grep -E "tsk|tsm" >> gpurun_out/r05w_ts.log || { cp gpurun_out/.keep_tsm.so gladsgp_amd/libgpfit.so; exit 1; }
  done
done
cp gpurun_out/.keep_tsm.so gladsgp_amd/libgpfit.so
cat gpurun_out/r05w_ts.log
