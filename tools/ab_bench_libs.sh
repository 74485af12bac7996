#!/bin/bash
# Same-box A/B of whole library builds on the C3 and C4 benches: each build in turn is copied
# over gladsgp_amd/libgpfit.so, two interleaved rounds.
#   tools/ab_bench_libs.sh TAG lib1.so lib2.so ...   -> gpurun_out/TAG.log
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=$1; shift
mkdir -p gpurun_out
cp gladsgp_amd/libgpfit.so gpurun_out/.libgpfit_keep.so
: > gpurun_out/$TAG.log
for rep in 1 2; do
  for lib in "$@"; do
    cp "$lib" gladsgp_amd/libgpfit.so
    for wl in ${AB_WORKLOADS:-c3 c4}; do
      st=10; [ $wl = c4 ] && st=5; [ $wl = c5 ] && st=5
      timeout -k 10 200 python bench.py --workload $wl --steps $st --warmup 2 --no-cpu > gpurun_out/${TAG}_one.log 2>&1 || { cat gpurun_out/${TAG}_one.log; cp gpurun_out/.libgpfit_keep.so gladsgp_amd/libgpfit.so; exit 1; }
      python -c "
import json
l=json.loads([x for x in open('gpurun_out/${TAG}_one.log').read().splitlines() if x.startswith('{')][-1])
r=l['roofline']
print('%-28s %s step %.3f ms  %.2fM pred/s  trmm %.4f ms/launch (%.1f TF/s, frac %.4f)' % ('$(basename $lib)', '$wl', l['ms_per_step'], l['value']/1e6, r['avg_launch_ms'], r['achieved'], r['frac']))
" >> gpurun_out/$TAG.log || exit 1
    done
  done
done
cp gpurun_out/.libgpfit_keep.so gladsgp_amd/libgpfit.so
cat gpurun_out/$TAG.log
