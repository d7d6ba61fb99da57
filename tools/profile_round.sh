#!/bin/bash
# Profile one bench preset on the GPU box: the bench line (with the CPU baseline), a rocprofv3
# kernel-trace summary of the same command, one SQ counter pass and the FETCH/WRITE passes for the
# HBM-traffic field.  Each GPU step has its own time limit; the script stops at the first failure.
#   TAG=r01_fft1 PRESET=gate_fft tools/profile_round.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01}
PRESET=${PRESET:-gate_fft}
B="--preset $PRESET"
timeout -k 10 300 python bench.py $B > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || { echo "bench failed"; tail -30 gpurun_out/bench_${TAG}.err; exit 1; }
cat gpurun_out/bench_${TAG}.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- python3 bench.py $B --no-cpu > gpurun_out/prof_${TAG}.log 2>&1 || { echo "rocprof stats failed"; tail -30 gpurun_out/prof_${TAG}.log; exit 1; }
find gpurun_out/prof_${TAG} -name '*kernel_stats.csv' -exec cp {} gpurun_out/${TAG}_kernel_stats.csv \;
head -6 gpurun_out/${TAG}_kernel_stats.csv | cut -c1-200
tail -1 gpurun_out/prof_${TAG}.log
timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT -d gpurun_out/pmc_sq_${TAG} -o run --output-format csv -- python3 bench.py $B --steps 2 --warmup 1 --no-cpu > gpurun_out/pmc_sq_${TAG}.log 2>&1 || { echo "pmc sq failed"; tail -20 gpurun_out/pmc_sq_${TAG}.log; exit 1; }
find gpurun_out/pmc_sq_${TAG} -name '*counter_collection.csv' -exec cp {} gpurun_out/${TAG}_pmc_sq.csv \;
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_${TAG} -o run --output-format csv -- python3 bench.py $B --steps 2 --warmup 1 --no-cpu > gpurun_out/pmc_fetch_${TAG}.log 2>&1 || { echo "pmc fetch failed"; tail -20 gpurun_out/pmc_fetch_${TAG}.log; exit 1; }
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write_${TAG} -o run --output-format csv -- python3 bench.py $B --steps 2 --warmup 1 --no-cpu > gpurun_out/pmc_write_${TAG}.log 2>&1 || { echo "pmc write failed"; tail -20 gpurun_out/pmc_write_${TAG}.log; exit 1; }
for d in pmc_fetch_${TAG} pmc_write_${TAG}; do f=$(find gpurun_out/$d -name '*counter_collection.csv' | head -1); mkdir -p gpurun_out/${d}_flat; cp "$f" gpurun_out/${d}_flat/run_counter_collection.csv; done
echo ALL_OK
