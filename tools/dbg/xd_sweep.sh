set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for xd in ${XDS:-0 2 4 8}; do
  export GPFIT_PP_XD=$xd
  timeout -k 10 120 python tools/prof_potrf.py 4096 8 1 | tail -1 | sed "s/^/xd=$xd /" >> gpurun_out/xd_time.log || exit 1
  timeout -k 10 120 python tools/prof_potrf.py 1024 6 32 | tail -1 | sed "s/^/xd=$xd /" >> gpurun_out/xd_time.log || exit 1
  timeout -k 10 120 python tools/dbg/pp_trace.py 4096 > gpurun_out/ppt_xd$xd.log 2>&1 || exit 1
done
