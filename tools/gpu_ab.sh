#!/bin/bash
# GPU box job: parity tests, then tools/ab_env.sh over $ENVS (see there).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/ab_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/ab_pytest.log; [ $rc -ne 0 ] && exit $rc
bash tools/ab_env.sh
