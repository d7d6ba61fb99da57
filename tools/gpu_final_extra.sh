#!/bin/bash
# On the GPU box: smoke() and the default bench exactly as the driver runs them, then the C2 (batch 1024) A/B over
# build_ab/* (pair kernel CTS 2 vs 4).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > gpurun_out/smoke_final.log 2>&1 || { tail -20 gpurun_out/smoke_final.log; exit 1; }
tail -1 gpurun_out/smoke_final.log
timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail gpurun_out/bench_default.err; exit 1; }
head -c 400 gpurun_out/bench_default.json; echo
BENCH_ARGS="--batch 1024" ROUNDS="1 2" timeout -k 10 400 bash tools/ab_run.sh || exit 1
echo ALL_OK
