#!/bin/bash
# On the GPU box: the squash parity tests on the in-tree library, then tools/sns_ab_libs.sh over build_ab/*.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_sns.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/sns_ab_tests.log 2>&1 || { tail -30 gpurun_out/sns_ab_tests.log; exit 1; }
tail -2 gpurun_out/sns_ab_tests.log
ROUNDS="${ROUNDS:-1 2}" timeout -k 10 900 bash tools/sns_ab_libs.sh
