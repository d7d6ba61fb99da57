#!/bin/bash
# On the GPU box: noise-squash throughput (tools/sns_bench.py, B = 1024) for every library variant in
# build_ab/* (tools/ab_build.sh), ROUNDS times.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out && export TMPDIR=/tmp
for round in ${ROUNDS:-1 2}; do
  for d in build_ab/*/; do
    n=$(basename $d)
    TFHE_HIP_LIB=$PWD/$d/libtfhe_hip.so timeout -k 10 200 python tools/sns_bench.py --batch 1024 --steps 2 > gpurun_out/sns_ab_$n.json 2>/dev/null || { echo "$n failed"; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/sns_ab_$n.json'));print('$n', 'round $round', d['value'], d['ms_per_batch'], d['decrypt_ok'])"
  done
done
echo ALL_OK
