"""Blind-rotate kernel time vs batch size for the latency kernel and the batch kernel (P-GATE),
measured with the library's HIP events; prints one JSON object.  Picks the crossover used as the
default of tfhe_hip_set_latency_batch.   python tools/latency_sweep.py"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tfhe_amd  # noqa: E402


def main():
    import torch
    params = tfhe_amd.Params.preset(tfhe_amd.PRESET_GATE)
    ck, sk = tfhe_amd.gen_keys(params, 0x7F4E0001)
    eng = tfhe_amd.Engine(params, 0).load_keys(sk)
    dev = torch.device("cuda", 0)
    res = {}
    for B in [1, 8, 64, 256, 257, 512, 768, 1024, 1280, 1536, 2048, 4096]:
        cts = ck.encrypt_bool(np.arange(B) % 2 == 0, seed=9)
        d_in = torch.from_numpy(cts.view(np.int64)).to(dev)
        d_lut = torch.from_numpy(eng.gate_lut().view(np.int64)).to(dev)
        d_out = torch.empty_like(d_in)
        row = {}
        for name, thr in (("latency", 1 << 30), ("batch", 0)):
            if name == "latency" and B > 2048:
                continue
            eng.set_latency_batch(thr)
            eng.pbs_async(d_in, d_lut, d_out)
            torch.cuda.synchronize()
            eng.timing(True)
            eng.timing_reset()
            reps = 3
            for _ in range(reps):
                eng.pbs_async(d_in, d_lut, d_out)
            torch.cuda.synchronize()
            eng.timing(False)
            ms, n = eng.timing_stats(0)
            row[name] = round(ms / max(n, 1), 3)
            ok = np.array_equal(ck.decrypt_bool(d_out.cpu().numpy().view(np.uint64)), np.arange(B) % 2 == 0)
            assert ok, (B, name)
        res[B] = row
        print(B, row, file=sys.stderr, flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
