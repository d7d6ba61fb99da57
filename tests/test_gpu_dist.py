"""Multi-rank engine path on the GPU (configs C2, C4's partition, C5): two processes, each
with its own tfhe_amd.Engine, in one torch.distributed group (gloo: both ranks share device 0 of a
one-GPU box, which RCCL does not allow).  Rank 0 generates and broadcasts the keys once; a global
batch is bootstrapped as per-rank contiguous shards and all_gathered; the result must equal a
single-rank run bit for bit and the CPU oracle on a sample that straddles the shard boundary; the C5
auction tree runs with every level sharded, as host arrays and device-resident (the level's tensors sliced,
launched and all_gathered on the device), bit-equal across ranks, forms and a single-rank run of the same
circuit shape (tests/gpu_dist_worker.py does the work).

The ranks are started as child processes (fork + exec of a fresh interpreter) of this pytest process.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _run_world(preset: str, tmp_path, world: int = 2, G: int = 1024, backend: str = "gloo"):
    port = _free_port()
    procs, outs = [], []
    for r in range(world):
        out = str(tmp_path / f"rank{r}.json")
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), DIST_BACKEND=backend)
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "gpu_dist_worker.py"), preset, out,
                                       str(G)],
                                      cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
        outs.append(out)
    logs = []
    try:
        for p in procs:
            logs.append(p.communicate(timeout=400)[0])
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for p, log in zip(procs, logs):
        assert p.returncode == 0, log[-3000:]
    return [json.load(open(o)) for o in outs]


@pytest.mark.parametrize("preset", ["gate_fft", "gate", "fhevm_fft"])
def test_world2_engines_shard_gather_bitexact(preset, tmp_path):
    res = _run_world(preset, tmp_path)
    r0 = res[0]
    assert r0["equal_single_rank"], r0
    assert r0["oracle_sample_ok"], r0
    assert r0["decrypt_ok"], r0
    if preset != "fhevm_fft":
        for r in res:
            assert r["c5_ok"], r
            assert r["c5_dev_ok"] and r["c5_dev_tensor"], r
        # the tree's comparisons really were split: each rank ran a share of the PBS, on both circuit forms
        assert all(r["c5_pbs_this_rank"] > 0 and r["c5_dev_pbs_this_rank"] > 0 for r in res)
        assert sum(r["c5_dev_pbs_this_rank"] for r in res) == r0["c5_single_pbs"]
        # the device-resident sharded tree: the same bits on every rank, as the host-array sharded tree and as a
        # single-rank run of the same circuit shape
        assert len({r["c5_dev_digest"] for r in res} | {r0["c5_host_digest"], r0["c5_single_digest"]}) == 1, res
    print({r["rank"]: {k: r[k] for k in r if k.endswith("_s") or k.endswith("_ms")} for r in res})


def test_world1_rccl_path(tmp_path):
    """The RCCL ("nccl" backend) code path on a one-GPU box: a world-1 communicator runs the key broadcast, the C2
    shard + all_gather and the C5 tree (host-array and device-resident forms, every level through sharded_map) on
    DEVICE buffers -- what the 8-GPU node runs per rank, minus the peers (gloo cannot host device tensors, and RCCL
    refuses two ranks on one device)."""
    r0 = _run_world("gate_fft", tmp_path, world=1, backend="nccl")[0]
    assert r0["backend"] == "nccl", r0
    assert r0["equal_single_rank"] and r0["oracle_sample_ok"] and r0["decrypt_ok"], r0
    assert r0["c5_ok"] and r0["c5_dev_ok"] and r0["c5_dev_tensor"], r0
    assert len({r0["c5_dev_digest"], r0["c5_host_digest"], r0["c5_single_digest"]}) == 1, r0
    print({k: r0[k] for k in r0 if k.endswith("_s") or k.endswith("_ms")})


def test_bench_under_torchrun_one_rank(tmp_path):
    """bench.py as the driver launches it for N > 1 (python -m torch.distributed.run ... bench.py --gpus N), with one
    rank: the process group comes up on RCCL and the key broadcast, barriers and max-over-ranks all_reduce run."""
    port = _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1", "--master-addr",
           "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"), "--gpus", "1", "--steps", "2",
           "--warmup", "1", "--batch", "1024", "--no-cpu"]
    p = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=400)
    assert p.returncode == 0, (p.stdout[-2000:], p.stderr[-3000:])
    line = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][-1])
    assert line["n_gpus"] == 1 and line["decrypt_ok"], line
    # the line records the process group bench.py really created (not a grep of the log)
    assert line["dist"] == {"backend": "nccl", "world_size": 1}, line.get("dist")
    assert line["key_broadcast_ms"] > 0, line
    print({k: line[k] for k in ("value", "ms_per_step", "n_gpus")})


def test_world2_c4_global_batch_65536(tmp_path):
    """C4's global batch (65,536 PBS, BASELINE.json configs[3]) through the world-2 engine path: 32,768 PBS per
    rank, gathered, equal to a single-rank run of all 65,536, decrypted, oracle-exact across the rank boundary."""
    res = _run_world("gate_fft", tmp_path, G=65536)
    r0 = res[0]
    assert r0["equal_single_rank"] and r0["decrypt_ok"] and r0["oracle_sample_ok"], r0
    assert 32767 in r0["oracle_sample"] and 32768 in r0["oracle_sample"]
    print({r["rank"]: r["sharded_s"] for r in res})
