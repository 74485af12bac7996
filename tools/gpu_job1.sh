set -o pipefail
cd /root/repo
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/bench1.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /root/repo/gpurun_out/prof1 -o run --output-format csv -- python3 /root/repo/bench.py --steps 5 --warmup 2 --no-cpu > /root/repo/gpurun_out/prof1.log 2>&1
rc=$?
cd /root/repo; tail -3 gpurun_out/smoke.log; cat gpurun_out/bench1.log | tail -5; exit $rc
