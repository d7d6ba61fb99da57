#!/bin/bash
# One GPU-box session for a kernel change: FFT64 parity tests, then the bench line at the metric config and at
# C2 (batch 1024), optionally the profile round.  Each GPU step has its own limit; stops at the first failure.
#   TAG=r03_x [TESTS="tests/test_gpu_fft.py ..."] [PROFILE=1] bash tools/gpu_step.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r03}
TESTS=${TESTS:-tests/test_gpu_fft.py}
timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -3 gpurun_out/${TAG}_tests.log
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 300 python bench.py --no-cpu ${BENCH_ARGS:-} > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "bench failed"; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_bench.json'));r=d['roofline'];print('BENCH', d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'], d['decrypt_ok'])"
  timeout -k 10 300 python bench.py --no-cpu --batch 1024 --steps 20 > gpurun_out/${TAG}_c2.json 2> gpurun_out/${TAG}_c2.err || { echo "c2 bench failed"; tail -20 gpurun_out/${TAG}_c2.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_c2.json'));r=d['roofline'];print('C2', d['value'], d['ms_per_step'], r['kernel_ms'], d['decrypt_ok'])"
fi
if [ "${PROFILE:-0}" = "1" ]; then
  TAG=${TAG} PRESET=gate_fft bash tools/profile_round.sh > gpurun_out/${TAG}_prof.log 2>&1 || { echo "profile failed"; tail -20 gpurun_out/${TAG}_prof.log; exit 1; }
  tail -6 gpurun_out/${TAG}_prof.log
fi
echo STEP_OK
