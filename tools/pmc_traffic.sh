#!/bin/bash
# HBM traffic per kernel from PMC counters (separate passes: FETCH_SIZE, WRITE_SIZE).
#   tools/pmc_traffic.sh [c3|c4|c5]   -> gpurun_out/pmc_traffic.json | pmc_traffic_c4.json
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
WL=${1:-c3}
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c -d $R/gpurun_out/pmc_${WL}_$c -o run --output-format csv -- python3 $R/bench.py --workload $WL --steps 2 --warmup 1 --no-cpu > $R/gpurun_out/pmc_${WL}_$c.log 2>&1 || exit 1
done
python3 - "$R" "$WL" <<'PY'
import csv, glob, json, sys, collections
R, WL = sys.argv[1], sys.argv[2]
means = collections.defaultdict(dict)
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    f = glob.glob(f"{R}/gpurun_out/pmc_{WL}_{c}/**/*counter_collection.csv", recursive=True)
    if not f:
        print("no counter csv for", c, glob.glob(f"{R}/gpurun_out/pmc_{c}/**/*", recursive=True)); continue
    rows = list(csv.DictReader(open(f[0])))
    agg = collections.defaultdict(list)
    for r in rows:
        agg[r["Kernel_Name"][:60]].append(float(r["Counter_Value"]))
    for k, v in agg.items():
        print(f"{c:11s} {k:50s} n={len(v):4d} mean={sum(v)/len(v):14.1f} (KB per dispatch)")
        key = k.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
        means[key.split("<")[0]][c] = sum(v) / len(v)     # trmm_pair_kernel<false> -> base name
# the dominant kernel's HBM-side bytes per launch for bench.py's roofline.traffic: FETCH_SIZE x2
# (gfx950 reports half the bytes of 16-B/lane streams, MI355X_MICROARCH.md HBM section) + WRITE
dom = "trmm_res_kernel" if WL == "c5" else "trmm_pair_kernel"
t = means.get(dom, {})
if t:
    if WL == "c3":
        # 6 launches per step since round 5 (the 1696-point tail runs merged with chunk 6)
        n, m, chunk, batch, launches = 4096, 100000, 16384, 1, 6
    elif WL == "c4":                     # C4: 32 GPs, n = 1024, 8192-point chunks
        n, m, chunk, batch, launches = 1024, 100000, 8192, 32, 13
    else:                                # C5: 64 PC GPs, n = 512, 13 launches per step
        n, m, chunk, batch, launches = 512, 100000, 7936, 64, 13
    L = 8.0 * n * (n + 1) / 2 * batch    # L^-1 lower triangles
    if dom == "trmm_pair_kernel":
        alg = L + 8.0 * n * m / launches * batch          # + the launch's mean Kt chunk
        alg_note = "L^-1 lower triangle(s) + the launch's mean Kt chunk"
    else:                                # K* is produced in LDS: test points in, mean/var out
        alg = L + (64.0 + 16.0 * batch) * m / launches
        alg_note = ("L^-1 lower triangles + the launch's mean test points (64 B) and mean/var "
                    "(16 B per prediction); K* never reaches memory.  The kernel's L^-1 loads "
                    "are 8 B per lane (128 B per 16-lane column): the x2 correction, calibrated "
                    "on 16-B/lane streams, is assumed to hold for them (uncalibrated width)")
    out = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes) of "
                     "`bench.py --steps 2 --warmup 1 --no-cpu`, MI355X (tools/pmc_traffic.sh)",
           "correction": "FETCH_SIZE x2 (gfx950 tallies 16-B/lane streams at half their bytes); "
                         "WRITE_SIZE as reported",
           "workload": WL, "m_chunk": chunk, "m": m, "n": n, "batch": batch,
           "kernels": {dom: {
               "fetch_kb_raw": t.get("FETCH_SIZE"), "write_kb": t.get("WRITE_SIZE"),
               "bytes_per_launch": 1024.0 * (2 * t.get("FETCH_SIZE", 0) + t.get("WRITE_SIZE", 0)),
               "algorithmic_bytes_per_launch": alg,
               "note": f"per-dispatch mean over the {launches} launches of a step; algorithmic = "
                       + alg_note}}}
    for k, v in means.items():
        if k != dom:
            out["kernels"][k] = {"fetch_kb_raw": v.get("FETCH_SIZE"), "write_kb": v.get("WRITE_SIZE")}
    name = "pmc_traffic.json" if WL == "c3" else f"pmc_traffic_{WL}.json"
    json.dump(out, open(f"{R}/gpurun_out/{name}", "w"), indent=1)
    print(dom, "bytes/launch", out["kernels"][dom]["bytes_per_launch"])
PY
