"""Noise-squashing throughput on one MI355X: B small-key P-FHEVM ciphertexts -> 128-bit LWEs
(k=2, N=2048, 2^24 x 3), inputs resident in HBM, timed with HIP events on torch's stream.
  python tools/sns_bench.py [--batch B] [--steps K]"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tfhe_amd  # noqa: E402
from tfhe_amd import sns as S  # noqa: E402


def log(msg):  # progress on stderr, flushed: a run that stalls shows how far it got
    print(f"[sns_bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=3)
    a = ap.parse_args()
    params = tfhe_amd.Params.preset(tfhe_amd.PRESET_FHEVM)
    log(f"start: batch {a.batch}, steps {a.steps}, TFHE_HIP_SNS_CHUNK={os.environ.get('TFHE_HIP_SNS_CHUNK')}")
    ck, sk = tfhe_amd.gen_keys(params, 0x7F4E0001)
    eng = tfhe_amd.Engine(params, 0).load_keys(sk)
    log("P-FHEVM keys loaded")
    sp = S.SnsParams.preset(0)
    t = time.time()
    key = S.SquashedKey(sp, 0x7F4E0001, ck.lwe_key)
    keygen_s = time.time() - t
    log(f"squash key generated in {keygen_s:.1f}s")
    sq = S.Squasher(sp, 0).load_key(key)
    log("squash key loaded")
    B = a.batch
    msgs = (np.arange(B) % 16).astype(np.uint64)
    small, _ = eng.ms_reduce(eng.keyswitch(ck.encrypt(msgs, 16, seed=5)))
    dev = torch.device("cuda:0")
    d_in = torch.from_numpy(small.view(np.int64)).to(dev)
    d_out = torch.empty((B, sp.k * sp.N + 1, 2), dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream(dev)
    log("inputs ready; warm-up squash")
    sq.squash_async(d_in, B, d_out, 16, s)
    torch.cuda.synchronize()
    log("warm-up done; timed squashes")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(a.steps):
        sq.squash_async(d_in, B, d_out, 16, s)
    e1.record(s)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.steps
    log(f"timed squashes done: {ms:.2f} ms per batch")
    ok = bool(np.array_equal(key.decrypt(d_out.cpu().numpy().view(np.uint64)), msgs))
    print(json.dumps({"metric": "noise squashes/s (P-FHEVM small key -> 128-bit LWE, k=2 N=2048 2^24x3)",
                      "value": round(B / (ms * 1e-3), 1), "ms_per_batch": round(ms, 2), "batch": B,
                      "product": "fft64-limbs, native 2^128 torus",
                      "sns_bsk_mb": round(key.bsk.nbytes / 1e6, 1), "keygen_s": round(keygen_s, 1),
                      "decrypt_ok": ok}), flush=True)


if __name__ == "__main__":
    main()
