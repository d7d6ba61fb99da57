#!/bin/bash
# On the GPU box: one LDS-utilisation counter pass per FFT64 preset (LDS-array cycles, LDS instruction issue and
# waits, VALU issue; summed over the chip) -> gpurun_out/<TAG>_lds_<preset>.csv.  Each pass under its own time limit.
#   TAG=r05j bash tools/lds_pmc.sh
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-lds}
for p in gate_fft fhevm_fft; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE -d gpurun_out/pmc_lds_${T}_$p -o run --output-format csv -- python3 bench.py --preset $p --steps 2 --warmup 1 --no-cpu > gpurun_out/pmc_lds_${T}_$p.log 2>&1 || { echo "pmc $p failed"; tail -5 gpurun_out/pmc_lds_${T}_$p.log; exit 1; }
  find gpurun_out/pmc_lds_${T}_$p -name '*counter_collection.csv' -exec cp {} gpurun_out/${T}_lds_$p.csv \;
  rm -rf gpurun_out/pmc_lds_${T}_$p
done
echo LDS_OK
