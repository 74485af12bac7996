#!/bin/bash
# A/B of trmm_res_kernel builds (lib x GPFIT_TRMM_RES mode) on C5, two interleaved rounds.
#   tools/ab_res2.sh TAG "lib1.so lib2.so" "1 2 0"  -> gpurun_out/TAG.log
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=$1; LIBS=$2; MODES=${3:-"1 0"}
cp gladsgp_amd/libgpfit.so gpurun_out/.libgpfit_keep.so
: > gpurun_out/$TAG.log
for rep in 1 2; do
  for lib in $LIBS; do
    cp "$lib" gladsgp_amd/libgpfit.so
    for res in $MODES; do
      GPFIT_TRMM_RES=$res timeout -k 10 200 python bench.py --workload c5 --steps 5 --warmup 2 --no-cpu > gpurun_out/${TAG}_one.log 2>&1 || { cat gpurun_out/${TAG}_one.log; cp gpurun_out/.libgpfit_keep.so gladsgp_amd/libgpfit.so; exit 1; }
      python -c "
import json
l=json.loads([x for x in open('gpurun_out/${TAG}_one.log').read().splitlines() if x.startswith('{')][-1])
r=l['roofline']; ph=l['phases_ms']
print('%-22s RES=$res c5 step %.3f ms  %.2fM pred/s  svd %.3f  predict %.3f  get_y %.3f ms  trmm %.4f ms/launch x %d (%.1f TF/s)' % ('$(basename $lib)', l['ms_per_step'], l['value']/1e6, ph['svd'], ph['predict'], ph['get_y'], r['avg_launch_ms'], r['launches'], r['achieved']))
" >> gpurun_out/$TAG.log || exit 1
    done
  done
done
cp gpurun_out/.libgpfit_keep.so gladsgp_amd/libgpfit.so
cat gpurun_out/$TAG.log
