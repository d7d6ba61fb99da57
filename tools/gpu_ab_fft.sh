set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_fft.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/ab1_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/ab1_tests.log; exit 1; }
tail -2 gpurun_out/ab1_tests.log
ROUNDS="1 2" timeout -k 10 600 bash tools/ab_run.sh || exit 1
echo AB_OK
