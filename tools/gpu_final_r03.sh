#!/bin/bash
# Round 3's evidence job (profiles/r03/): the whole GPU suite + smoke, the C3 bench with its CPU
# baseline, rocprofv3 kernel trace + stats of a short bench and its step timeline, PMC passes
# (HBM traffic of the C3 and C4 benches -> pmc_traffic*.json, MFMA busy), the factorisation's
# dataflow trace, the C4 / fit / latency workloads, the self-launched two-rank bench on the one
# GPU, and the same-box factorisation A/B against round 2's library.  Each step has its own
# time limit; the first failure ends the job.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-f3}
R=$(pwd)
mkdir -p gpurun_out
step() { echo "== $1 $(date +%T)"; }
step pytest
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_pytest.log; [ $rc -ne 0 ] && exit $rc
step smoke
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit 1
tail -1 gpurun_out/${TAG}_smoke.log
step bench
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/${TAG}_bench.log 2>&1 || exit 1
tail -1 gpurun_out/${TAG}_bench.log | cut -c1-300
step rocprof
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_prof -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu > $R/gpurun_out/${TAG}_prof.log 2>&1 || exit 1
python3 $R/tools/step_timeline.py $R/gpurun_out/${TAG}_prof/run_kernel_trace.csv > $R/gpurun_out/${TAG}_timeline.txt || exit 1
step pmc
bash $R/tools/pmc_traffic.sh c3 > $R/gpurun_out/${TAG}_pmc.txt 2>&1 || exit 1
tail -1 $R/gpurun_out/${TAG}_pmc.txt
bash $R/tools/pmc_traffic.sh c4 > $R/gpurun_out/${TAG}_pmc_c4.txt 2>&1 || exit 1
tail -1 $R/gpurun_out/${TAG}_pmc_c4.txt
bash $R/tools/pmc_mfma.sh > $R/gpurun_out/${TAG}_pmc_mfma.txt 2>&1 || exit 1
cd $R
step pptrace
timeout -k 10 120 python tools/dbg/pp_trace.py 4096 > gpurun_out/${TAG}_pptrace.txt 2>&1 || exit 1
step c4
timeout -k 10 300 python bench.py --workload c4 --steps 5 --warmup 2 > gpurun_out/${TAG}_c4.log 2>&1 || exit 1
tail -1 gpurun_out/${TAG}_c4.log | cut -c1-200
step fit
timeout -k 10 400 python bench.py --workload fit > gpurun_out/${TAG}_fit.log 2>&1 || exit 1
tail -1 gpurun_out/${TAG}_fit.log | cut -c1-200
step latency
timeout -k 10 400 python bench.py --workload latency --latency-points 10 --warmup 2 > gpurun_out/${TAG}_latency.log 2>&1 || exit 1
tail -1 gpurun_out/${TAG}_latency.log | cut -c1-300
step bench_n2
timeout -k 10 400 python bench.py --gpus 2 --share-gpu --steps 5 --warmup 2 --no-cpu > gpurun_out/${TAG}_bench_n2.log 2>&1 || exit 1
grep '^{' gpurun_out/${TAG}_bench_n2.log | cut -c1-300
if [ -f _ab/libgpfit_r02.so ]; then
step ab_r02
timeout -k 10 200 python tools/ab_libs.py _ab/libgpfit_r02.so gladsgp_amd/libgpfit.so > gpurun_out/${TAG}_ab_r02.log 2>&1 || exit 1
tail -4 gpurun_out/${TAG}_ab_r02.log
fi
step done
step ab_spec
bash tools/ab_mcmc_spec.sh ${TAG}_ab_spec 2 3 > /dev/null || exit 1
cat gpurun_out/${TAG}_ab_spec.log
step end
