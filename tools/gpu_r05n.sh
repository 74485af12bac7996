# Round-5 evidence, part 1: PMC traffic (C3, C4), MFMA busy (C3), kernel-trace stats + timeline
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
R0=$(pwd)
step() { echo "== $1 $(date +%T)"; }
step pmc_c3
bash tools/pmc_traffic.sh c3 > gpurun_out/r05n_pmc_c3.log 2>&1 || { tail -5 gpurun_out/r05n_pmc_c3.log; exit 1; }
tail -2 gpurun_out/r05n_pmc_c3.log
step pmc_c4
bash tools/pmc_traffic.sh c4 > gpurun_out/r05n_pmc_c4.log 2>&1 || { tail -5 gpurun_out/r05n_pmc_c4.log; exit 1; }
tail -2 gpurun_out/r05n_pmc_c4.log
step mfma_c3
bash tools/pmc_mfma.sh c3 > gpurun_out/r05n_pmc_mfma_c3.txt 2>&1 || { tail -5 gpurun_out/r05n_pmc_mfma_c3.txt; exit 1; }
head -12 gpurun_out/r05n_pmc_mfma_c3.txt
step rocprof_c3
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R0/gpurun_out/r05n_prof -o run --output-format csv -- python3 $R0/bench.py --steps 5 --warmup 2 --no-cpu > $R0/gpurun_out/r05n_prof.log 2>&1 || exit 1
python3 $R0/tools/step_timeline.py $R0/gpurun_out/r05n_prof/run_kernel_trace.csv > $R0/gpurun_out/r05n_timeline.txt || exit 1
head -14 $R0/gpurun_out/r05n_timeline.txt
step rocprof_c4
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R0/gpurun_out/r05n_prof_c4 -o run --output-format csv -- python3 $R0/bench.py --workload c4 --steps 3 --warmup 1 --no-cpu > $R0/gpurun_out/r05n_prof_c4.log 2>&1 || exit 1
step end
