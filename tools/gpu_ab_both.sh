#!/bin/bash
# On the GPU box: P-GATE and P-FHEVM bench A/B over build_ab/* (no parity tests: build options of the shipped code)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out && export TMPDIR=/tmp
ROUNDS="1 2" timeout -k 10 500 bash tools/ab_run.sh || exit 1
BENCH_ARGS="--preset fhevm_fft" ROUNDS="1 2" timeout -k 10 600 bash tools/ab_run.sh || exit 1
echo AB_OK
