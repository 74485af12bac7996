#!/bin/bash
# Same-box A/B of TRMM block->tile mappings (kXcdPanels = 0 / 4 / 8): C3 + C4 bench times
# (tools/ab_bench_libs.sh) and the TRMM's FETCH_SIZE per launch at C3 for each build.
#   tools/ab_trmm_map.sh TAG lib...    -> gpurun_out/TAG.log, gpurun_out/TAG_fetch.log
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
TAG=$1; shift
bash tools/ab_bench_libs.sh "$TAG" "$@" || exit 1
cp gladsgp_amd/libgpfit.so gpurun_out/.libgpfit_keep2.so
: > gpurun_out/${TAG}_fetch.log
for lib in "$@"; do
  cp "$lib" gladsgp_amd/libgpfit.so
  b=$(basename "$lib" .so)
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE -d "$R/gpurun_out/pmcab_$b" -o run --output-format csv -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu > "$R/gpurun_out/pmcab_$b.log" 2>&1) || { cp gpurun_out/.libgpfit_keep2.so gladsgp_amd/libgpfit.so; exit 1; }
  python3 - "$R/gpurun_out/pmcab_$b" "$b" >> gpurun_out/${TAG}_fetch.log <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
v = [float(r["Counter_Value"]) for r in csv.DictReader(open(f)) if "trmm_pair" in r["Kernel_Name"]]
print(f"{sys.argv[2]:12s} trmm FETCH_SIZE x2 per launch: {2 * sum(v) / len(v) / 1e6:.3f} GB "
      f"(mean of {len(v)} launches; max {2 * max(v) / 1e6:.3f})")
PY
done
cp gpurun_out/.libgpfit_keep2.so gladsgp_amd/libgpfit.so
cat gpurun_out/${TAG}_fetch.log
