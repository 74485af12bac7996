set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/kmaj_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/kmaj_pytest.log; [ $rc -ne 0 ] && exit $rc
bash tools/ab_libs.sh cur kmaj || exit 1
cp gpurun_out/ab_libs.log gpurun_out/ab_kmaj_c3.log
bash tools/pmc_lds.sh > gpurun_out/pmc_lds_kmaj.txt 2>&1; grep "trmm\|cross" gpurun_out/pmc_lds_kmaj.txt
