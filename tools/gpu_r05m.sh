set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 250 --timeout-method thread > gpurun_out/r05m_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r05m_pytest.log; [ $rc -ne 0 ] && exit $rc
AB_WORKLOADS="c4" timeout -k 10 600 bash tools/ab_bench_libs.sh r05m_umap _ab/libgpfit_cur.so _ab/libgpfit_umap.so || exit 1
