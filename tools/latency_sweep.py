"""Blind-rotate kernel time vs batch size for the latency kernel and the batch kernel, measured with
the library's HIP events; prints one JSON object.  Picks the crossover used as the default of
tfhe_hip_set_latency_batch.   python tools/latency_sweep.py [gate|fhevm|gate_fft|fhevm_fft] [B,B,...]"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tfhe_amd  # noqa: E402


def main():
    import torch
    which = sys.argv[1] if len(sys.argv) > 1 else "gate"
    fhevm = which.startswith("fhevm")
    preset = {"gate": tfhe_amd.PRESET_GATE, "fhevm": tfhe_amd.PRESET_FHEVM, "gate_fft": tfhe_amd.PRESET_GATE_FFT,
              "fhevm_fft": tfhe_amd.PRESET_FHEVM_FFT}[which]
    params = tfhe_amd.Params.preset(preset)
    sizes = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else \
        [1, 8, 64, 256, 257, 512, 768, 1024, 1280, 1536, 2048, 4096]
    ck, sk = tfhe_amd.gen_keys(params, 0x7F4E0001)
    eng = tfhe_amd.Engine(params, 0).load_keys(sk)
    dev = torch.device("cuda", 0)
    res = {}
    for B in sizes:
        want = np.arange(B) % (16 if fhevm else 2)
        cts = ck.encrypt(want, 16, seed=9) if fhevm else ck.encrypt_bool(want == 0, seed=9)
        lut = eng.generate_accumulator(lambda m: m, 16) if fhevm else eng.gate_lut()
        d_in = torch.from_numpy(cts.view(np.int64)).to(dev)
        d_lut = torch.from_numpy(lut.view(np.int64)).to(dev)
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
            o = d_out.cpu().numpy().view(np.uint64)
            ok = np.array_equal(ck.decrypt(o, 16), want) if fhevm else np.array_equal(ck.decrypt_bool(o), want == 0)
            assert ok, (B, name)
        res[B] = row
        print(B, row, file=sys.stderr, flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
