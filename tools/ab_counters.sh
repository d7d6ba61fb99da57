#!/bin/bash
# On the GPU box: SQ counter passes (one rocprofv3 --pmc run each) for every variant in build_ab/*, so two
# kernels' wait / instruction / LDS profiles can be compared side by side.  Summaries: gpurun_out/abc_<variant>_*.csv
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
PASSES=${PASSES:-"SQ_WAVE_CYCLES,SQ_INSTS_VALU,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_WAIT_INST_LDS,SQ_INSTS_LDS,SQ_LDS_BANK_CONFLICT,SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM,SQ_ACTIVE_INST_LDS,SQ_ACTIVE_INST_ANY,SQ_BUSY_CYCLES,SQ_LDS_IDX_ACTIVE,SQ_INSTS_SALU,GRBM_GUI_ACTIVE"}
for d in build_ab/*/; do
  n=$(basename $d)
  k=0
  for p in $PASSES; do
    k=$((k+1))
    TFHE_HIP_LIB=$PWD/$d/libtfhe_hip.so timeout -s KILL 120 rocprofv3 --pmc ${p//,/ } -d gpurun_out/abc_${n}_$k -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu ${BENCH_ARGS:-} > gpurun_out/abc_${n}_$k.log 2>&1 || { echo "$n pass $k failed"; tail -5 gpurun_out/abc_${n}_$k.log; exit 1; }
    find gpurun_out/abc_${n}_$k -name '*counter_collection.csv' -exec cp {} gpurun_out/abc_${n}_$k.csv \;
    rm -rf gpurun_out/abc_${n}_$k
  done
  python - "$n" <<'PY'
import csv, glob, sys
n = sys.argv[1]
agg = {}
for f in sorted(glob.glob(f"gpurun_out/abc_{n}_*.csv")):
    for r in csv.DictReader(open(f)):
        if "blind_rotate" not in r["Kernel_Name"]:
            continue
        agg.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
print(n, {k: round(sum(v) / len(v) / 1e6, 2) for k, v in sorted(agg.items())}, "(millions, per launch)")
PY
done
