"""Packing-keyswitch throughput on one MI355X (ML2048 preset: 2048 LWEs of dim 2048 per GLWE).
Times pack_async on a torch stream with HIP events; prints one JSON line.
  python tools/pks_bench.py [--glwes G] [--steps K]"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tfhe_amd import compression as C  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--glwes", type=int, default=8)
    ap.add_argument("--steps", type=int, default=5)
    a = ap.parse_args()
    pp = C.PksParams.preset(C.PKS_PRESET_ML2048)
    in_key = np.random.default_rng(5).integers(0, 2, pp.in_dim).astype(np.uint64)
    t = time.time()
    ck = C.CompressionKey(pp, 0x7F4E0001, in_key)
    keygen_s = time.time() - t
    packer = C.Packer(pp, 0).load_key(ck)
    count = a.glwes * pp.lwe_per_glwe
    lwes = np.random.default_rng(1).integers(0, 2 ** 63, size=(count, pp.in_dim + 1), dtype=np.uint64)
    dev = torch.device("cuda:0")
    d_in = torch.from_numpy(lwes.view(np.int64)).to(dev)
    d_out = torch.empty((a.glwes, pp.glwe_len), dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream(dev)
    packer.pack_async(d_in, count, d_out, s)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(a.steps):
        packer.pack_async(d_in, count, d_out, s)
    e1.record(s)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.steps
    K = pp.in_dim * pp.level
    macs = count * K * pp.glwe_len
    ref = packer.pack(lwes[-pp.lwe_per_glwe:])[0]
    same = bool(np.array_equal(d_out[-1].cpu().numpy().view(np.uint64), ref))
    print(json.dumps({"metric": "packing keyswitch LWE/s (ML2048: dim 2048 -> GLWE k=1 N=2048, 2 x 2^14)",
                      "lwe_per_s": round(count / (ms * 1e-3), 1), "glwe_per_s": round(a.glwes / (ms * 1e-3), 2),
                      "ms_per_call": round(ms, 3), "lwes_per_call": count,
                      "gemm_tmac_per_s": round(macs / (ms * 1e-3) / 1e12, 3),
                      "pksk_mb": round(ck.pksk.nbytes / 1e6, 1), "keygen_s": round(keygen_s, 2),
                      "consistent": same}), flush=True)


if __name__ == "__main__":
    main()
