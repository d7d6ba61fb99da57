#!/bin/bash
# End-of-round evidence on the final tree: the whole -m gpu suite (SUITE), the profile set of both FFT64 presets and of
# C3 (C3=1: bench.py --config c3, 32,768 PBS per launch)
# (PROFILES; tools/profile_round.sh: rocprofv3 kernel stats, SQ / FETCH / WRITE / mix counter passes -> <TAG>_roofline.json
# tagged with this tree's source_id, then the bench line with the CPU baseline reading it), and EXTRA: C2, the squash
# profile (tools/gpu_sns_prof.sh) and C5 (tools/c5_bench.py).  Stops at the first failure.  Split over two calls to stay
# inside gpurun's limit:  SUITE=1 PROFILES=1 EXTRA=0 ... ; SUITE=0 PROFILES=0 EXTRA=1 ...
#   TAG=r05z bash tools/gpu_final.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r04z}
if [ "${SUITE:-1}" = "1" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 420 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_full.log 2>&1 || { echo "gpu tests failed"; grep -E "FAILED|Error|passed|failed" gpurun_out/${TAG}_full.log | tail -20; exit 1; }
  grep -E "passed|C5 |C4 on" gpurun_out/${TAG}_full.log | tail -6
fi
if [ "${PROFILES:-1}" = "1" ]; then
  TAG=${TAG} PRESET=gate_fft bash tools/profile_round.sh > gpurun_out/${TAG}_prof.log 2>&1 || { echo "gate profile failed"; tail -20 gpurun_out/${TAG}_prof.log; exit 1; }
  tail -3 gpurun_out/${TAG}_prof.log
  TAG=${TAG}_fhevm PRESET=fhevm_fft bash tools/profile_round.sh > gpurun_out/${TAG}_fhevm_prof.log 2>&1 || { echo "fhevm profile failed"; tail -20 gpurun_out/${TAG}_fhevm_prof.log; exit 1; }
  tail -3 gpurun_out/${TAG}_fhevm_prof.log
fi
if [ "${C3:-1}" = "1" ]; then  # BASELINE configs[2]: 4096 FheUint8 x 8 LUTs = 32,768 PBS per launch (bench.py --config c3)
  TAG=${TAG}_c3 PRESET=gate_fft ARGS="--config c3" BATCH=32768 MIX=0 bash tools/profile_round.sh > gpurun_out/${TAG}_c3_prof.log 2>&1 || { echo "c3 profile failed"; tail -20 gpurun_out/${TAG}_c3_prof.log; exit 1; }
  tail -3 gpurun_out/${TAG}_c3_prof.log
fi
if [ "${EXTRA:-1}" = "1" ]; then  # C2 (batch 1024), the squash bench + kernel stats, C5 timed
  timeout -k 10 300 python -u bench.py --batch 1024 --steps 10 --warmup 3 --no-cpu > gpurun_out/${TAG}_c2_bench.json 2> gpurun_out/${TAG}_c2_bench.err || { echo "C2 bench failed"; tail gpurun_out/${TAG}_c2_bench.err; exit 1; }
  TAG=${TAG}_sns bash tools/gpu_sns_prof.sh > gpurun_out/${TAG}_sns_prof.log 2>&1 || { echo "squash profile failed"; tail gpurun_out/${TAG}_sns_prof.log; exit 1; }
  timeout -k 10 300 python -u tools/c5_bench.py > gpurun_out/${TAG}_c5_bench.json 2> gpurun_out/${TAG}_c5_bench.err || { echo "C5 bench failed"; tail gpurun_out/${TAG}_c5_bench.err; exit 1; }
  tail -c 300 gpurun_out/${TAG}_c2_bench.json; head -c 300 gpurun_out/${TAG}_c5_bench.json; echo
fi
echo FINAL_OK
