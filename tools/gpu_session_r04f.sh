#!/bin/bash
# r04f: seeded-key GPU test + FFT parity, then the P-FHEVM A/B variants in build_ab/ (two rounds)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_seeded.py tests/test_gpu_fft.py tests/test_gpu_fft2k.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04f_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r04f_tests.log; exit 1; }
tail -2 gpurun_out/r04f_tests.log
ROUNDS="1 2" BENCH_ARGS="--preset fhevm_fft" timeout -k 10 800 bash tools/ab_run.sh || exit 1
echo SESSION_OK
