set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 250 --timeout-method thread > gpurun_out/r05f_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r05f_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/prof_pca.py > gpurun_out/r05f_prof_pca.log 2>&1 || exit 1
grep -E "init_model|gemm\(" gpurun_out/r05f_prof_pca.log | head -20
timeout -k 10 900 bash tools/ab_bench_libs.sh r05f_ab _ab/libgpfit_pk_new.so _ab/libgpfit_tabexp_ts.so || exit 1
