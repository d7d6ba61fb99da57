#!/bin/bash
# On the GPU box: bench each variant in build_ab/* (blind-rotate kernel ms).  Ablation variants
# produce wrong outputs on purpose (decrypt_ok False); a variant that crashes stops the run.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for round in ${ROUNDS:-1}; do
  for d in build_ab/${ONLY:-*}/; do
    n=$(basename $d)
    rm -f gpurun_out/ab_$n.json
    TFHE_HIP_LIB=$PWD/$d/libtfhe_hip.so timeout -k 10 300 python bench.py ${BENCH_ARGS:-} --steps 5 --warmup 2 --no-cpu > gpurun_out/ab_$n.json 2>/dev/null
    rc=$?
    if [ ! -s gpurun_out/ab_$n.json ]; then echo "$n CRASHED rc=$rc"; exit 1; fi
    python -c "import json;d=json.load(open('gpurun_out/ab_$n.json'));print('$n', 'round $round', 'PBS/s', d['value'], 'br_ms', d['roofline']['kernel_ms'], 'ks_ms', d['keyswitch_ms'], 'ok', d['decrypt_ok'])"
  done
done
