#!/bin/bash
# One GPU-box session: parity tests, a 2-rank rehearsal of the distributed bench path on one GPU
# (gloo, same device), and HBM counter passes for the blind-rotate kernel.  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
    bench.py --gpus 2 --steps 3 --warmup 1 --batch 1024 --dist-backend gloo --same-device > gpurun_out/bench_rehearsal2.log 2> gpurun_out/bench_rehearsal2.err || { echo "rehearsal failed"; tail -30 gpurun_out/bench_rehearsal2.err; exit 1; }
cat gpurun_out/bench_rehearsal2.log
if [ "${PMC:-1}" = "1" ]; then
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu > gpurun_out/pmc_fetch.log 2>&1 || { echo "pmc fetch failed"; tail -20 gpurun_out/pmc_fetch.log; exit 1; }
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu > gpurun_out/pmc_write.log 2>&1 || { echo "pmc write failed"; tail -20 gpurun_out/pmc_write.log; exit 1; }
fi
echo ALL_OK
