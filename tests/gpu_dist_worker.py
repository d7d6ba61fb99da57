"""One rank of the multi-rank engine check (driven by tests/test_gpu_dist.py; not a test module).

Every rank runs its own tfhe_amd.Engine (all on device 0 on a one-GPU box; one GPU per rank on a
node) in a torch.distributed group:
  1. rank 0 generates the key set and broadcasts BSK / KSK (+ the P-FHEVM modulus-switch zeros) once;
     every rank loads them from its device buffers (tfhe_hip_load_keys_device) — SURVEY §8e;
  2. one global batch (C2: 1024 PBS) is bootstrapped as contiguous shards, one per rank, and
     all_gathered (tfhe_amd.dist.sharded_map); rank 0 checks the gathered batch bit-for-bit against
     a single-rank run of the whole batch, against the CPU oracle on a sample, and by decryption;
  3. (P-GATE) the C5 auction tree (256 FheUint32 bids, 8 levels) with every level sharded over the
     ranks and the winners all_gathered between levels.

  RANK=r WORLD_SIZE=w MASTER_ADDR=127.0.0.1 MASTER_PORT=p [DIST_BACKEND=nccl] python tests/gpu_dist_worker.py PRESET OUT_JSON [G]

DIST_BACKEND (default gloo: two ranks sharing device 0, which RCCL refuses) = nccl runs the same steps over RCCL: the
key broadcast and every all_gather on device buffers (one rank per GPU; on a one-GPU box a world-1 communicator).

G (default 1024, C2) sets the global batch of step 2; G = 65536 is C4's global batch (BASELINE.json configs[3]),
checked at both sides of the rank boundary; step 3 (C5) runs only at the default G.
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import tfhe_amd  # noqa: E402
from tfhe_amd.dist import broadcast_keys, sharded_map  # noqa: E402

KEY_SEED = 0x7F4E0001


def main(preset_name: str, out_path: str, G: int = 1024) -> int:
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    backend = os.environ.get("DIST_BACKEND", "gloo")
    dev = torch.device("cuda", 0 if backend == "gloo" else int(os.environ.get("LOCAL_RANK", "0")))
    torch.cuda.set_device(dev)
    if backend == "nccl":
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    else:
        dist.init_process_group(backend, rank=rank, world_size=world)
    res = {"rank": rank, "world": world, "preset": preset_name, "backend": dist.get_backend()}
    try:
        preset = {"gate_fft": tfhe_amd.PRESET_GATE_FFT, "gate": tfhe_amd.PRESET_GATE,
                  "fhevm_fft": tfhe_amd.PRESET_FHEVM_FFT}[preset_name]
        params = tfhe_amd.Params.preset(preset)
        L = tfhe_amd.lib()
        import ctypes
        bsk_len = L.tfhe_hip_bsk_len(ctypes.byref(params))
        ksk_len = L.tfhe_hip_ksk_len(ctypes.byref(params))
        fhevm = params.order == 1
        # 1. keys on rank 0, broadcast once
        if rank == 0:
            ck, sk = tfhe_amd.gen_keys(params, KEY_SEED)
            bsk = torch.from_numpy(sk.bsk.view(np.int64).copy())
            ksk = torch.from_numpy(sk.ksk.view(np.int64).copy())
            zeros = torch.from_numpy(sk.ms_zeros.view(np.int64).copy()) if fhevm else None
        else:
            ck, _ = tfhe_amd.gen_keys(params, KEY_SEED, with_server_key=False)
            bsk = torch.empty(bsk_len, dtype=torch.int64)
            ksk = torch.empty(ksk_len, dtype=torch.int64)
            zeros = torch.empty((tfhe_amd.MS_FHEVM["count"], params.n + 1), dtype=torch.int64) if fhevm else None
        if backend == "nccl":   # RCCL broadcasts device buffers
            bsk, ksk = bsk.to(dev), ksk.to(dev)
            zeros = zeros.to(dev) if fhevm else None
        res["bcast_ms"] = broadcast_keys(bsk, ksk, src=0)
        if fhevm:
            dist.broadcast(zeros, src=0)
        eng = tfhe_amd.Engine(params, dev.index)
        eng.load_keys_device(bsk.to(dev), ksk.to(dev))
        if fhevm:
            eng.load_ms_key(zeros.cpu().numpy().view(np.uint64))

        # 2. one global batch (C2 by default, C4 at G = 65536), sharded over the ranks and gathered
        rng = np.random.default_rng(0xC0FFEE02)
        if fhevm:
            msgs = rng.integers(0, 16, G).astype(np.uint64)
            cts = ck.encrypt(msgs, 16, seed=0xC0FFEE02, stream0=0)
            lut = eng.generate_accumulator(lambda m: (3 * m + 1) % 16, 16)
        else:
            bits = rng.integers(0, 2, G).astype(bool)
            cts = ck.encrypt_bool(bits, seed=0xC0FFEE02, stream0=0)
            lut = eng.gate_lut()
        t0 = time.time()
        out = sharded_map(torch.from_numpy(cts.view(np.int64)),
                          lambda s: torch.from_numpy(eng.pbs(s.numpy().view(np.uint64), lut).view(np.int64)))
        res["sharded_s"] = time.time() - t0
        out = out.numpy().view(np.uint64)
        if rank == 0:
            single = eng.pbs(cts, lut)
            res["equal_single_rank"] = bool(np.array_equal(out, single))
            if fhevm:
                res["decrypt_ok"] = bool(np.array_equal(ck.decrypt(out, 16), (3 * msgs + 1) % 16))
            else:
                res["decrypt_ok"] = bool(np.array_equal(ck.decrypt_bool(out), bits))
            from oracle import oracle as O
            prm = O.params(preset)
            keys = O.Keys(prm, KEY_SEED)
            bounds = [G * r // world for r in range(1, world)]
            sel = np.array(sorted({0, 1, G - 1} | {b + d for b in bounds for d in (-1, 0, 1)}))  # both sides of each boundary
            ref = O.pbs_batch(prm, keys, cts[sel], lut[None])   # P-FHEVM: with the same MS zeros (seeded)
            res["oracle_sample"] = sel.tolist()
            res["oracle_sample_ok"] = bool(np.array_equal(out[sel], ref))

        # 3. C5 auction tree, every level sharded over the ranks
        if not fhevm and G == 1024:
            from tfhe_amd import integer as I
            from tfhe_amd.auction import max_tree
            v = np.random.default_rng(5).integers(0, 2**32, 256, dtype=np.uint64)
            v[77] = v[200] = np.uint64(2**32 - 3)
            c = I.Circuit(eng)
            bids = I.FheUint.encrypt(c, ck, v, 32, seed=0xB1D, stream0=0)
            t0 = time.time()
            mx, idx = max_tree(c, bids, group=dist.group.WORLD)
            res["c5_s"] = time.time() - t0
            res["c5_ok"] = int(mx.decrypt(ck)[0]) == 2**32 - 3 and int(idx.decrypt(ck)[0]) == 77
            res["c5_pbs_this_rank"] = c.pbs_count
            # the device-resident tree (round 5): every level sliced, launched and gathered as device tensors
            import hashlib

            def digest(*arrs):
                h = hashlib.sha256()
                for a in arrs:
                    h.update(np.ascontiguousarray(a.cpu().numpy() if isinstance(a, torch.Tensor) else a).view(np.uint8))
                return h.hexdigest()

            cd = I.Circuit(eng, device=str(dev))
            bd = I.FheUint.encrypt(cd, ck, v, 32, seed=0xB1D, stream0=0)
            torch.cuda.synchronize()
            t0 = time.time()
            mxd, idxd = max_tree(cd, bd, group=dist.group.WORLD)
            torch.cuda.synchronize()
            res["c5_dev_s"] = time.time() - t0
            res["c5_dev_tensor"] = isinstance(mxd.bits, torch.Tensor) and mxd.bits.is_cuda
            res["c5_dev_ok"] = int(mxd.decrypt(ck)[0]) == 2**32 - 3 and int(idxd.decrypt(ck)[0]) == 77
            res["c5_dev_pbs_this_rank"] = cd.pbs_count
            res["c5_dev_digest"] = digest(mxd.bits, idxd.bits)
            res["c5_host_digest"] = digest(mx.bits.view(np.int64), idx.bits.view(np.int64))
            if rank == 0:
                # single rank, same circuit shape: a shard of P/world pairs costs what P pairs cost at world x the
                # launch-round size (Circuit.carry_block's model is linear in the batch), so the block sizes agree
                c1 = I.Circuit(eng, device=str(dev), round_size=world * eng.round_size)
                b1 = I.FheUint.encrypt(c1, ck, v, 32, seed=0xB1D, stream0=0)
                mx1, idx1 = max_tree(c1, b1)
                res["c5_single_digest"] = digest(mx1.bits, idx1.bits)
                res["c5_single_pbs"] = c1.pbs_count
        eng.close()
    finally:
        with open(out_path, "w") as f:
            json.dump(res, f)
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 1024))
