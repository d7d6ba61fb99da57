#!/bin/bash
# On the GPU box: noise-squash bench + rocprofv3 kernel stats of the in-tree library (TAG names the outputs).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-sns}
timeout -k 10 200 python -u tools/sns_bench.py --batch 1024 --steps 2 > gpurun_out/${T}_bench.json 2>gpurun_out/${T}_bench.err || { tail gpurun_out/${T}_bench.err; exit 1; }
cat gpurun_out/${T}_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${T} -o run --output-format csv -- python3 tools/sns_bench.py --batch 1024 --steps 1 > gpurun_out/prof_${T}.log 2>&1 || { tail -5 gpurun_out/prof_${T}.log; exit 1; }
find gpurun_out/prof_${T} -name "*kernel_stats.csv" -exec cp {} gpurun_out/${T}_kernel_stats.csv \;
cut -d, -f1-4 gpurun_out/${T}_kernel_stats.csv | head -6
echo ALL_OK
