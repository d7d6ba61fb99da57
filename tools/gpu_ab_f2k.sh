#!/bin/bash
# On the GPU box: the N = 2048 FFT64 parity tests on the in-tree library, then P-FHEVM bench A/B over build_ab/*.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_fft2k.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/f2k_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/f2k_tests.log; exit 1; }
tail -2 gpurun_out/f2k_tests.log
BENCH_ARGS="--preset fhevm_fft" ROUNDS="1 2" timeout -k 10 700 bash tools/ab_run.sh || exit 1
echo AB_OK
