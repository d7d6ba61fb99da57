#!/bin/bash
# On the GPU box: latency-kernel vs batch-kernel blind-rotate time per batch size (HIP events) for both FFT64 presets.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-lat}
timeout -k 10 300 python -u tools/latency_sweep.py gate_fft 1,8,64,128,256,320,384,512,768,1024 > gpurun_out/${T}_gate.json 2> gpurun_out/${T}_gate.err || { tail gpurun_out/${T}_gate.err; exit 1; }
cat gpurun_out/${T}_gate.json
timeout -k 10 300 python -u tools/latency_sweep.py fhevm_fft 1,8,64,128,256,384,512,640,768,1024 > gpurun_out/${T}_fhevm.json 2> gpurun_out/${T}_fhevm.err || { tail gpurun_out/${T}_fhevm.err; exit 1; }
cat gpurun_out/${T}_fhevm.json
echo ALL_OK
