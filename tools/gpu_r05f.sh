set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 250 --timeout-method thread > gpurun_out/r05f_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r05f_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/ab_xcd_queues.py > gpurun_out/r05f_xcd_queues.log 2>&1 || { cat gpurun_out/r05f_xcd_queues.log; exit 1; }
cat gpurun_out/r05f_xcd_queues.log
timeout -k 10 900 bash tools/ab_bench_libs.sh r05f_ab _ab/libgpfit_pk_new.so _ab/libgpfit_fs.so _ab/libgpfit_xq.so _ab/libgpfit_pmix1.so _ab/libgpfit_pmix2.so _ab/libgpfit_pmix3.so || exit 1
