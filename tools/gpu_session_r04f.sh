#!/bin/bash
# r04f: seeded-key GPU test, FFT parity, the C5 tests (host and device-resident circuits) and the C5 bench in both
# modes, then the P-FHEVM A/B variants in build_ab/ (two rounds).  Every GPU step has its own limit; stops at the
# first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_seeded.py tests/test_gpu_fft.py tests/test_gpu_fft2k.py "tests/test_gpu_configs.py::test_c5_device_resident_equals_host" -m gpu -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04f_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r04f_tests.log; exit 1; }
grep -E "C5 fft64|passed|failed" gpurun_out/r04f_tests.log | tail -4
timeout -k 10 300 python -u tools/c5_bench.py > gpurun_out/r04f_c5_device.json 2> gpurun_out/r04f_c5_device.err || { echo "c5 device bench failed"; tail -10 gpurun_out/r04f_c5_device.err; exit 1; }
cut -c1-300 gpurun_out/r04f_c5_device.json
timeout -k 10 300 python -u tools/c5_bench.py --host > gpurun_out/r04f_c5_host.json 2> gpurun_out/r04f_c5_host.err || { echo "c5 host bench failed"; tail -10 gpurun_out/r04f_c5_host.err; exit 1; }
cut -c1-300 gpurun_out/r04f_c5_host.json
ROUNDS="1 2" BENCH_ARGS="--preset fhevm_fft" timeout -k 10 800 bash tools/ab_run.sh || exit 1
echo SESSION_OK
