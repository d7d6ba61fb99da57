#!/bin/bash
# On the GPU box: parity tests on the in-tree library (TESTS, default the FFT64 parity + exact-arbiter files), then
# the bench A/B over build_ab/* (tools/ab_build.sh) for each preset in PRESETS, ROUNDS interleaved rounds each.
#   TESTS="tests/test_gpu_fft.py" PRESETS="gate_fft fhevm_fft" ROUNDS="1 2" bash tools/gpu_ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out && export TMPDIR=/tmp
TESTS=${TESTS-tests/test_gpu_fft.py tests/test_gpu_fft2k.py tests/test_gpu_exact.py tests/test_gpu_parity.py}
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/ab_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" gpurun_out/ab_tests.log | head; tail -5 gpurun_out/ab_tests.log; exit 1; }
  tail -1 gpurun_out/ab_tests.log
fi
for p in ${PRESETS:-gate_fft fhevm_fft}; do
  BENCH_ARGS="--preset $p" ROUNDS="${ROUNDS:-1 2}" timeout -k 10 700 bash tools/ab_run.sh || exit 1
done
echo AB_OK
