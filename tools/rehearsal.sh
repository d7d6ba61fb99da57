#!/bin/bash
# Two-rank rehearsal of bench.py's distributed path on ONE GPU (both ranks on device 0, gloo for the
# barrier / max-over-ranks / key broadcast): weak scaling (the metric's mode) and --global-batch strong
# scaling.  Records the rank-0 JSON lines under gpurun_out/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=${TAG:-rehearsal2}
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 \
    bench.py --gpus 2 --steps 3 --warmup 1 --batch 2048 --dist-backend gloo --same-device --no-cpu \
    > gpurun_out/${TAG}_weak.json 2> gpurun_out/${TAG}_weak.err || { echo "weak rehearsal failed"; tail -30 gpurun_out/${TAG}_weak.err; exit 1; }
cat gpurun_out/${TAG}_weak.json
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29532 \
    bench.py --gpus 2 --steps 3 --warmup 1 --global-batch 4096 --dist-backend gloo --same-device --no-cpu \
    > gpurun_out/${TAG}_strong.json 2> gpurun_out/${TAG}_strong.err || { echo "strong rehearsal failed"; tail -30 gpurun_out/${TAG}_strong.err; exit 1; }
cat gpurun_out/${TAG}_strong.json
echo ALL_OK
