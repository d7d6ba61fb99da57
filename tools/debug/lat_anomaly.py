"""Time the latency kernels around the batch sizes that looked slow (B = 256 at N = 2048, 1024 at N = 1024)."""
import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import tfhe_amd
for preset, Bs in ((tfhe_amd.PRESET_FHEVM_FFT, (224, 255, 256, 257, 288)), (tfhe_amd.PRESET_GATE_FFT, (960, 1023, 1024, 1025))):
    ck, sk = tfhe_amd.gen_keys(tfhe_amd.Params.preset(preset), 0x7F4E0001)
    eng = tfhe_amd.Engine(ck.params, 0); eng.load_keys(sk); eng.set_latency_batch(1 << 20)
    p = ck.params
    lut = eng.generate_accumulator(lambda m: m, 16)
    for B in Bs:
        cts = np.random.default_rng(B).integers(0, 2**63, (B, p.n + 1), dtype=np.uint64)
        eng.blind_rotate(cts, lut)
        ts = []
        for _ in range(5):
            t = time.time(); eng.blind_rotate(cts, lut); ts.append((time.time() - t) * 1e3)
        print(preset, B, " ".join(f"{x:.2f}" for x in ts), flush=True)
