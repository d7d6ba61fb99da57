#!/bin/bash
# On the GPU box: the noise-squash bench, rocprofv3 kernel stats, and the counter passes of the squash kernels
# (SQ issue / waits, FETCH_SIZE, WRITE_SIZE, instruction mix -- one rocprofv3 run each), folded by
# tools/roofline_summary.py into gpurun_out/<TAG>_roofline.json; then the batch-tiling A/B: a 1024 batch run as
# two sequential 512-ciphertext chunks (TFHE_HIP_SNS_CHUNK=512), whose per-CMUX intermediates fit the 256 MB
# Infinity Cache, with its own bench line and FETCH/WRITE passes.  Each GPU step has its own time limit; the script
# stops at the first failure.
#   TAG=r05_sns bash tools/gpu_sns_prof.sh
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-sns}
CMD="python3 tools/sns_bench.py --batch 1024 --steps 1"
timeout -k 10 200 python -u tools/sns_bench.py --batch 1024 --steps 3 > gpurun_out/${T}_bench.json 2>gpurun_out/${T}_bench.err || { tail gpurun_out/${T}_bench.err; exit 1; }
cat gpurun_out/${T}_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${T} -o run --output-format csv -- $CMD > gpurun_out/prof_${T}.log 2>&1 || { tail -5 gpurun_out/prof_${T}.log; exit 1; }
find gpurun_out/prof_${T} -name "*kernel_stats.csv" -exec cp {} gpurun_out/${T}_kernel_stats.csv \;
cut -d, -f1-4 gpurun_out/${T}_kernel_stats.csv | head -6
pmc() {  # pmc NAME COUNTERS... : one counter pass of the squash command
  local n=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" -d gpurun_out/pmc_${n}_${T} -o run --output-format csv -- $CMD > gpurun_out/pmc_${n}_${T}.log 2>&1 || { echo "pmc $n failed"; tail -5 gpurun_out/pmc_${n}_${T}.log; return 1; }
  find gpurun_out/pmc_${n}_${T} -name '*counter_collection.csv' -exec cp {} gpurun_out/${T}_pmc_${n}.csv \;
}
pmc sq SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS GRBM_GUI_ACTIVE || exit 1
pmc fetch FETCH_SIZE || exit 1
pmc write WRITE_SIZE || exit 1
pmc mix SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_SALU || exit 1
BATCH=1024 python tools/roofline_summary.py $T gpurun_out/${T}_kernel_stats.csv gpurun_out/${T}_pmc_sq.csv gpurun_out/${T}_pmc_fetch.csv gpurun_out/${T}_pmc_write.csv gpurun_out/${T}_pmc_mix.csv gpurun_out/${T}_roofline.json || { echo "summary failed"; exit 1; }
# tiling A/B: the same 1024 batch in two 512 chunks
export TFHE_HIP_SNS_CHUNK=512
timeout -k 10 200 python -u tools/sns_bench.py --batch 1024 --steps 3 > gpurun_out/${T}_chunk512_bench.json 2>gpurun_out/${T}_chunk512_bench.err || { tail gpurun_out/${T}_chunk512_bench.err; exit 1; }
cat gpurun_out/${T}_chunk512_bench.json
T0=$T; T=${T0}_chunk512
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${T} -o run --output-format csv -- $CMD > gpurun_out/prof_${T}.log 2>&1 || { tail -5 gpurun_out/prof_${T}.log; exit 1; }
find gpurun_out/prof_${T} -name "*kernel_stats.csv" -exec cp {} gpurun_out/${T}_kernel_stats.csv \;
pmc fetch FETCH_SIZE || exit 1
pmc write WRITE_SIZE || exit 1
BATCH=512 python tools/roofline_summary.py $T gpurun_out/${T}_kernel_stats.csv /dev/null gpurun_out/${T}_pmc_fetch.csv gpurun_out/${T}_pmc_write.csv gpurun_out/${T}_roofline.json || { echo "summary failed"; exit 1; }
# the raw rocprofv3 directories (per-launch traces of 918 x 3 launches) stay on the box: gpurun copies back <= 64 MiB
rm -rf gpurun_out/prof_${T0}* gpurun_out/pmc_*_${T0}*
echo ALL_OK
