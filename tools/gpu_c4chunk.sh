set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/c1_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/c1_pytest.log; [ $rc -ne 0 ] && exit $rc
bash tools/pmc_traffic.sh c4 > gpurun_out/c1_pmc_c4.txt 2>&1 || exit 1
tail -1 gpurun_out/c1_pmc_c4.txt
timeout -k 10 300 python bench.py --workload c4 --steps 5 --warmup 2 > gpurun_out/c1_c4.log 2>&1 || exit 1
tail -1 gpurun_out/c1_c4.log | cut -c1-250
timeout -k 10 300 python bench.py --workload c4 --m-chunk 4096 --steps 5 --warmup 2 --no-cpu > gpurun_out/c1_c4_4096.log 2>&1 || exit 1
tail -1 gpurun_out/c1_c4_4096.log | cut -c1-250
