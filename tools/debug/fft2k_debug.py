"""Localize an FFT2k blind-rotation mismatch: LUT init only, then one non-trivial CMUX."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import tfhe_amd
from oracle import oracle as O
prm = O.params(3)
ck, sk = tfhe_amd.gen_keys(tfhe_amd.Params.preset(tfhe_amd.PRESET_FHEVM_FFT), 0x7F4E0001)
keys = O.Keys(prm, 0x7F4E0001)
eng = tfhe_amd.Engine(ck.params, 0)
eng.load_keys(sk)
rng = np.random.default_rng(1)
lut = O.lut_from_table(2048, 16, [(m * 5 + 3) % 16 for m in range(16)], (1 << 63) // 16)
cts = np.zeros((4, 919), dtype=np.uint64)
cts[:, 918] = rng.integers(0, 2**64 - 1, 4, dtype=np.uint64)
cts[1, 0] = np.uint64(1 << 51) * np.uint64(3)      # one CMUX with a = 3 (odd)
cts[2, 5] = np.uint64(1 << 51) * np.uint64(1000)   # one CMUX with a = 1000
cts[3, :918] = rng.integers(0, 2**64 - 1, 918, dtype=np.uint64)
acc = eng.blind_rotate(cts, lut)
for i in range(4):
    ref = O.blind_rotate_fft(prm, keys, cts[i], lut)
    d = np.nonzero(acc[i] != ref)[0]
    print(i, "mismatches", len(d), d[:10], "A-part" if len(d) and d[0] < 2048 else "")
    if len(d):
        print("   dev", acc[i][d[:4]], "ref", ref[d[:4]], "diff", (acc[i][d[:4]] - ref[d[:4]]))
os.makedirs("gpurun_out", exist_ok=True)
np.save("gpurun_out/f2k_dbg_acc.npy", acc)
np.save("gpurun_out/f2k_dbg_cts.npy", cts)
Z = eng.fft_fwd(sk.bsk.reshape(-1, 2048)[:8])
np.save("gpurun_out/f2k_dbg_bskf.npy", Z)
