set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
timeout -k 10 300 python -u -m pytest tests/test_gpu_c3.py tests/test_gpu_c4.py tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread > gpurun_out/trmv_pytest.log 2>&1 || { tail -20 gpurun_out/trmv_pytest.log; exit 1; }
tail -1 gpurun_out/trmv_pytest.log
cp gladsgp_amd/libgpfit.so gpurun_out/.keep.so
for name in snake trmv snake trmv; do
  cp _ab/libgpfit_$name.so gladsgp_amd/libgpfit.so
  rm -rf $R/gpurun_out/tp_$name
  (cd /tmp && TMPDIR=/tmp timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/tp_$name -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu > $R/gpurun_out/tp_$name.log 2>&1) || exit 1
  echo "== $name"; python3 tools/step_timeline.py gpurun_out/tp_$name/run_kernel_trace.csv | grep -i "trmv\|span\|starts" || exit 1
done
cp gpurun_out/.keep.so gladsgp_amd/libgpfit.so
