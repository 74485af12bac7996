#!/bin/bash
# Round 4 follow-up job: C3 re-sweep of the cross-covariance stream's CU reservation after the
# factorisation changes, then C4 on this box: bench, MFMA busy + effective clock (PMC), HBM
# traffic of the TRMM (FETCH/WRITE, separate passes) -- the box-to-box spread question.
#   tools/gpu_r04c.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-r04c}
R=$(pwd)
mkdir -p gpurun_out
step() { echo "== $1 $(date +%T)"; }
step pytest_sub
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_dist.py tests/test_gpu_rccl.py -x -v -m gpu --timeout 250 --timeout-method thread > gpurun_out/${TAG}_pytest_sub.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_pytest_sub.log; [ $rc -ne 0 ] && exit $rc
step fact_cus
timeout -k 10 200 python tools/prof_fact_cus.py > gpurun_out/${TAG}_fact_cus.log 2>&1 || exit 1
cat gpurun_out/${TAG}_fact_cus.log
step fit
timeout -k 10 400 python bench.py --workload fit > gpurun_out/${TAG}_fit.log 2>&1 || exit 1
grep '^{' gpurun_out/${TAG}_fit.log | cut -c1-300
step sweep_aux
FRS="0 16 32" bash tools/sweep_aux_cus.sh ${TAG}_sweep_aux > /dev/null || exit 1
cat gpurun_out/${TAG}_sweep_aux.log
step sweep_cross_start
FRS="0" CSS="0 0.2 0.6" bash tools/sweep_aux_cus.sh ${TAG}_sweep_cs > /dev/null || exit 1
cat gpurun_out/${TAG}_sweep_cs.log
step c4
timeout -k 10 300 python bench.py --workload c4 --steps 5 --warmup 2 > gpurun_out/${TAG}_c4.log 2>&1 || exit 1
grep '^{' gpurun_out/${TAG}_c4.log | cut -c1-250
step c4_aux_chunks
for rep in 1 2; do
  for v in "predict -1" "fit_predict 1" "fit_predict 2"; do
    set -- $v
    timeout -k 10 200 python bench.py --workload c4 --steps 5 --warmup 2 --c4-path $1 --aux-chunks $2 > gpurun_out/${TAG}_c4_ab.tmp 2>&1 || exit 1
    echo "path=$1 aux_chunks=$2 $(grep '^{' gpurun_out/${TAG}_c4_ab.tmp | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(round(r["value"]/1e6,2), "M/s", round(r["ms_per_step"],2), "ms")')" | tee -a gpurun_out/${TAG}_c4_aux_chunks.log
  done
done
step pmc_c4
bash tools/pmc_mfma.sh c4 > gpurun_out/${TAG}_pmc_mfma_c4.txt 2>&1 || exit 1
grep -E "trmm|cross|pp_kernel" gpurun_out/${TAG}_pmc_mfma_c4.txt
step pmc_c3
bash tools/pmc_mfma.sh c3 > gpurun_out/${TAG}_pmc_mfma_c3.txt 2>&1 || exit 1
grep -E "trmm|cross|pp_kernel" gpurun_out/${TAG}_pmc_mfma_c3.txt
step traffic_c4
bash tools/pmc_traffic.sh c4 > gpurun_out/${TAG}_pmc_traffic_c4.txt 2>&1 || exit 1
tail -3 gpurun_out/${TAG}_pmc_traffic_c4.txt
step traffic_c3
bash tools/pmc_traffic.sh c3 > gpurun_out/${TAG}_pmc_traffic_c3.txt 2>&1 || exit 1
tail -3 gpurun_out/${TAG}_pmc_traffic_c3.txt
step end
