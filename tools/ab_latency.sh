#!/bin/bash
# On the GPU box: latency-kernel PBS time per batch for every variant in build_ab/* on both FFT64 presets
# (tools/latency_sweep_fft.sh with BATCHES, default 1,64,256).  Each step has its own time limit.
cd "${GRAFT_REPO_ROOT:-.}"
for d in build_ab/${ONLY:-*}/; do
  n=$(basename $d)
  for p in gate fhevm; do
    echo "== $n $p"
    TFHE_HIP_LIB=$PWD/$d/libtfhe_hip.so PRESET=$p BATCHES=${BATCHES:-1,64,256} timeout -k 10 240 bash tools/latency_sweep_fft.sh 2>&1 | grep "B=" || { echo "$n $p failed"; exit 1; }
  done
done
