#!/bin/bash
# Round-6 GPU job runner: tools/gpu_r06.sh TAG STEP...  (each step under its own time limit;
# stops at the first failing step).  Logs to gpurun_out/r06_TAG_*.
set -o pipefail
tag=$1; shift
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; echo "== $name ($(date +%T))"; timeout -k 10 "$lim" "$@" > "gpurun_out/r06_${tag}_${name}.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 "gpurun_out/r06_${tag}_${name}.log"; return $rc; }
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
for step in "$@"; do
  case $step in
    t_*) f=${step#t_}; run "$step" 600 $PYT "tests/test_gpu_${f}.py" || exit $? ;;
    gpu) run gpu 1100 $PYT -m gpu tests || exit $? ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
    bench) run bench 400 python -u bench.py || exit $? ;;
    c4) run c4 400 python -u bench.py --workload c4 || exit $? ;;
    c5) run c5 400 python -u bench.py --workload c5 || exit $? ;;
    c5q) run c5q 300 python -u bench.py --workload c5 --no-cpu --steps 5 --warmup 2 || exit $? ;;
    fit) run fit 400 python -u bench.py --workload fit || exit $? ;;
    prof_c5) run prof_c5 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r06_${tag}_prof_c5 -o c5 -- python -u bench.py --workload c5 --no-cpu --steps 5 --warmup 2 || exit $? ;;
    field_ab) run field_ab 300 python -u tools/field_ab.py || exit $? ;;
    c4q) run c4q 300 python -u bench.py --workload c4 --no-cpu --steps 5 --warmup 2 || exit $? ;;
    c3q) run c3q 300 python -u bench.py --no-cpu --steps 10 --warmup 3 || exit $? ;;
    ab_fit) run ab_fit 900 bash tools/ab_fit_libs.sh r06_ab_fit_inner _ab/libgpfit_old.so _ab/libgpfit_new.so _ab/libgpfit_inchain.so || exit $? ;;
    ab_trmm) AB_WORKLOADS="c3 c4 c5" run ab_trmm 1000 bash tools/ab_bench_libs.sh r06_ab_trmm_inner _ab/libgpfit_pre_trmm.so _ab/libgpfit_trmm_persist.so || exit $? ;;
    ab_diag) AB_WORKLOADS="c4 c5" run ab_diag 900 bash tools/ab_bench_libs.sh r06_ab_diag_inner _ab/libgpfit_base.so _ab/libgpfit_diag1.so _ab/libgpfit_diag2.so || exit $? ;;
    pmc_c5) run pmc_c5_traffic 700 bash tools/pmc_traffic.sh c5 && run pmc_c5_mfma 400 bash tools/pmc_mfma.sh c5 || exit $? ;;
    ab_zpre) AB_WORKLOADS="c3 c4 c5" run ab_zpre 1000 bash tools/ab_bench_libs.sh r06_ab_zpre_inner _ab/libgpfit_base.so _ab/libgpfit_zpre.so || exit $? ;;
    ab_res) run ab_res 900 bash tools/ab_res.sh r06_ab_res_inner || exit $? ;;
    pmc_res) run pmc_res 600 bash tools/pmc_res.sh r06_pmc_res || exit $? ;;
    ab_res2) run ab_res2 1100 bash tools/ab_res2.sh r06_ab_res2_inner "${AB_LIBS:-_ab/libgpfit_narrow.so}" "${AB_MODES:-2 1}" || exit $? ;;
    prof_c3) run prof_c3 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r06_${tag}_prof_c3 -o c3 -- python -u bench.py --no-cpu --steps 10 --warmup 3 || exit $? ;;
    lat) run lat 300 python -u bench.py --workload latency || exit $? ;;
    ab_cross) AB_WORKLOADS="c3 c4" run ab_cross 1000 bash tools/ab_bench_libs.sh r06_ab_cross_inner _ab/libgpfit_crossbase.so _ab/libgpfit_crossnt.so || exit $? ;;
    t_sched) run t_sched 600 $PYT tests/test_gpu_sched.py tests/test_gpu_c3.py tests/test_gpu_c4.py || exit $? ;;
    ab_spec) run ab_spec 1000 bash -c 'for S in ${AB_SPECS:-2 3 4 4 3 2}; do echo "spec $S"; GPFIT_MCMC_SPEC=$S timeout -k 10 240 python -u bench.py --workload fit --no-cpu | tail -1 || exit 1; done' || exit $? ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
