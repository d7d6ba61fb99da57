#!/bin/bash
# On the GPU box: one rocprofv3 counter pass per A/B variant in build_ab/* (tools/ab_build.sh), the bench preset's
# blind-rotate kernel rows summarised by tools/sq_summary.py -> gpurun_out/ab_pmc_<variant>_<pass>.csv.
#   PRESET=gate_fft PASSES="sq lds" bash tools/ab_pmc.sh
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out && export TMPDIR=/tmp
P=${PRESET:-gate_fft}
pmc_of() {
  case $1 in
    sq) echo "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" ;;
    lds) echo "SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_INSTS_VMEM SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_INSTS_FLAT SQ_WAVES GRBM_GUI_ACTIVE" ;;
    mix) echo "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_SALU" ;;
    fetch) echo "FETCH_SIZE" ;;
  esac
}
for d in build_ab/${ONLY:-*}/; do
  n=$(basename $d)
  for pass in ${PASSES:-sq}; do
    out=gpurun_out/pmc_ab_${n}_$pass
    TFHE_HIP_LIB=$PWD/$d/libtfhe_hip.so timeout -s KILL 120 rocprofv3 --pmc $(pmc_of $pass) -d $out -o run --output-format csv -- python3 bench.py --preset $P --steps 2 --warmup 1 --no-cpu > $out.log 2>&1 || { echo "pmc $n $pass failed"; tail -5 $out.log; exit 1; }
    f=$(find $out -name '*counter_collection.csv' | head -1)
    python3 tools/sq_summary.py "$f" > gpurun_out/ab_pmc_${n}_$pass.txt 2>&1 || cp "$f" gpurun_out/ab_pmc_${n}_$pass.csv
    cp "$f" gpurun_out/ab_pmc_${n}_$pass.csv
    rm -rf $out
    echo "== $n $pass"; cat gpurun_out/ab_pmc_${n}_$pass.txt
  done
done
echo PMC_OK
