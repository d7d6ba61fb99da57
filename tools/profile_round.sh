#!/bin/bash
# Profile one bench preset on the GPU box: a rocprofv3 kernel-trace summary of the bench command, one SQ
# counter pass, the FETCH/WRITE passes for the HBM-traffic field and an SQ instruction-mix pass; then
# tools/roofline_summary.py folds them into gpurun_out/<TAG>_roofline.json tagged with the tree's source_id,
# and finally the bench line itself (with the CPU baseline) reads that summary (bench.py uses a profile under
# profiles/ only while its source_id matches its own).  Each GPU step has its own time
# limit; the script stops at the first failure.
#   TAG=r02_fft1 PRESET=gate_fft tools/profile_round.sh
#   TAG=r06_c3 PRESET=gate_fft ARGS="--config c3" BATCH=32768 tools/profile_round.sh   (BASELINE configs[2]: the
#   summary's batch is the launch's PBS count, 8 x 4096)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r02}
PRESET=${PRESET:-gate_fft}
B="--preset $PRESET ${ARGS:-}"
BENCH=${BENCH:-1}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- python3 bench.py $B --no-cpu > gpurun_out/prof_${TAG}.log 2>&1 || { echo "rocprof stats failed"; tail -30 gpurun_out/prof_${TAG}.log; exit 1; }
find gpurun_out/prof_${TAG} -name '*kernel_stats.csv' -exec cp {} gpurun_out/${TAG}_kernel_stats.csv \;
head -6 gpurun_out/${TAG}_kernel_stats.csv | cut -c1-200
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS GRBM_GUI_ACTIVE -d gpurun_out/pmc_sq_${TAG} -o run --output-format csv -- python3 bench.py $B --steps 2 --warmup 1 --no-cpu > gpurun_out/pmc_sq_${TAG}.log 2>&1 || { echo "pmc sq failed"; tail -20 gpurun_out/pmc_sq_${TAG}.log; exit 1; }
find gpurun_out/pmc_sq_${TAG} -name '*counter_collection.csv' -exec cp {} gpurun_out/${TAG}_pmc_sq.csv \;
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_${TAG} -o run --output-format csv -- python3 bench.py $B --steps 2 --warmup 1 --no-cpu > gpurun_out/pmc_fetch_${TAG}.log 2>&1 || { echo "pmc fetch failed"; tail -20 gpurun_out/pmc_fetch_${TAG}.log; exit 1; }
find gpurun_out/pmc_fetch_${TAG} -name '*counter_collection.csv' -exec cp {} gpurun_out/${TAG}_pmc_fetch.csv \;
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write_${TAG} -o run --output-format csv -- python3 bench.py $B --steps 2 --warmup 1 --no-cpu > gpurun_out/pmc_write_${TAG}.log 2>&1 || { echo "pmc write failed"; tail -20 gpurun_out/pmc_write_${TAG}.log; exit 1; }
find gpurun_out/pmc_write_${TAG} -name '*counter_collection.csv' -exec cp {} gpurun_out/${TAG}_pmc_write.csv \;
MIXCSV=""
if [ "${MIX:-1}" = "1" ]; then
  if timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_SALU -d gpurun_out/pmc_mix_${TAG} -o run --output-format csv -- python3 bench.py $B --steps 2 --warmup 1 --no-cpu > gpurun_out/pmc_mix_${TAG}.log 2>&1; then
    find gpurun_out/pmc_mix_${TAG} -name '*counter_collection.csv' -exec cp {} gpurun_out/${TAG}_pmc_mix.csv \;
    MIXCSV=gpurun_out/${TAG}_pmc_mix.csv
  else
    echo "mix pass failed (optional)"; tail -5 gpurun_out/pmc_mix_${TAG}.log
  fi
fi
python tools/roofline_summary.py $TAG gpurun_out/${TAG}_kernel_stats.csv gpurun_out/${TAG}_pmc_sq.csv gpurun_out/${TAG}_pmc_fetch.csv gpurun_out/${TAG}_pmc_write.csv $MIXCSV gpurun_out/${TAG}_roofline.json || { echo "summary failed"; exit 1; }
# the bench line LAST, with the summary placed under profiles/ of this box's copy, so bench.py picks up the counters
# of this very build (same source_id) -- round 4's P-FHEVM line ran before its profile existed and carried nulls
if [ "$BENCH" = "1" ]; then
  cp gpurun_out/${TAG}_roofline.json profiles/${TAG}_roofline.json
  timeout -k 10 300 python bench.py $B > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || { echo "bench failed"; tail -30 gpurun_out/bench_${TAG}.err; exit 1; }
  cat gpurun_out/bench_${TAG}.json
fi
rm -rf gpurun_out/prof_${TAG} gpurun_out/pmc_*_${TAG}   # raw rocprofv3 directories: the summaries above are kept
echo ALL_OK
