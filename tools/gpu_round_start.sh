#!/bin/bash
# First GPU session of a round, in two parts (each fits one gpurun call; every GPU step has its own limit,
# the script stops at the first failure):
#   PART=1: the whole -m gpu suite, then the noise-squash bench and its rocprofv3 kernel summary, then the C5 timing
#   PART=2: the profile set of both FFT64 presets (tools/profile_round.sh: bench line, kernel stats, SQ and
#           FETCH/WRITE counter passes -> <TAG>_roofline.json tagged with this tree's source_id)
#   TAG=r04 PART=1 bash tools/gpu_round_start.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r04}
if [ "${PART:-1}" = "1" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 420 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_full.log 2>&1 || { echo "gpu tests failed"; grep -E "FAILED|Error|passed|failed" gpurun_out/${TAG}_full.log | tail -20; exit 1; }
  grep -E "passed|C5 |C4 on" gpurun_out/${TAG}_full.log | tail -6
  timeout -k 10 200 python -u tools/sns_bench.py --batch 1024 --steps 2 > gpurun_out/${TAG}_sns_bench.json 2> gpurun_out/${TAG}_sns_bench.err || { echo "sns bench failed"; tail -10 gpurun_out/${TAG}_sns_bench.err; exit 1; }
  cat gpurun_out/${TAG}_sns_bench.json
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_sns -o run --output-format csv -- python3 tools/sns_bench.py --batch 1024 --steps 1 > gpurun_out/prof_${TAG}_sns.log 2>&1 || { echo "sns profile failed"; tail -5 gpurun_out/prof_${TAG}_sns.log; exit 1; }
  find gpurun_out/prof_${TAG}_sns -name '*kernel_stats.csv' -exec cp {} gpurun_out/${TAG}_sns_kernel_stats.csv \;
  cut -c1-120 gpurun_out/${TAG}_sns_kernel_stats.csv | head -8
  timeout -k 10 300 python -u tools/c5_bench.py > gpurun_out/${TAG}_c5_bench.json 2> gpurun_out/${TAG}_c5_bench.err || { echo "c5 bench failed"; tail -10 gpurun_out/${TAG}_c5_bench.err; exit 1; }
  cut -c1-400 gpurun_out/${TAG}_c5_bench.json
else
  TAG=${TAG} PRESET=gate_fft bash tools/profile_round.sh > gpurun_out/${TAG}_prof.log 2>&1 || { echo "gate profile failed"; tail -20 gpurun_out/${TAG}_prof.log; exit 1; }
  tail -4 gpurun_out/${TAG}_prof.log
  TAG=${TAG}_fhevm PRESET=fhevm_fft bash tools/profile_round.sh > gpurun_out/${TAG}_fhevm_prof.log 2>&1 || { echo "fhevm profile failed"; tail -20 gpurun_out/${TAG}_fhevm_prof.log; exit 1; }
  tail -4 gpurun_out/${TAG}_fhevm_prof.log
fi
echo ALL_OK
