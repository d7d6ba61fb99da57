#!/bin/bash
# Full GPU-box pass: parity tests, the default bench line, a rocprofv3 kernel-trace summary of the
# same bench command, and separate PMC passes (FETCH_SIZE / WRITE_SIZE) for the HBM-traffic field.
# Each GPU step has its own time limit; the script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01}
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/gpu_tests.log; exit 1; }
  tail -3 gpurun_out/gpu_tests.log
fi
timeout -k 10 600 python bench.py > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || { echo "bench failed"; tail -30 gpurun_out/bench_${TAG}.err; exit 1; }
cat gpurun_out/bench_${TAG}.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- python3 bench.py --no-cpu > gpurun_out/prof_${TAG}.log 2>&1 || { echo "rocprof stats failed"; tail -30 gpurun_out/prof_${TAG}.log; exit 1; }
find gpurun_out/prof_${TAG} -name '*kernel_stats.csv' -exec cp {} gpurun_out/${TAG}_kernel_stats.csv \;
head -5 gpurun_out/${TAG}_kernel_stats.csv
tail -1 gpurun_out/prof_${TAG}.log
if [ "${PMC:-1}" = "1" ]; then
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu > gpurun_out/pmc_fetch.log 2>&1 || { echo "pmc fetch failed"; tail -20 gpurun_out/pmc_fetch.log; exit 1; }
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu > gpurun_out/pmc_write.log 2>&1 || { echo "pmc write failed"; tail -20 gpurun_out/pmc_write.log; exit 1; }
fi
echo ALL_OK
