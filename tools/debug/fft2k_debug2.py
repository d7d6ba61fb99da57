import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import tfhe_amd
from oracle import oracle as O
ck, sk = tfhe_amd.gen_keys(tfhe_amd.Params.preset(tfhe_amd.PRESET_FHEVM_FFT), 0x7F4E0001)
eng = tfhe_amd.Engine(ck.params, 0)
eng.load_keys(sk)
rng = np.random.default_rng(1)
cts = np.zeros((4, 919), dtype=np.uint64)
cts[:, 918] = rng.integers(0, 2**64 - 1, 4, dtype=np.uint64)
cts[1, 0] = np.uint64(1 << 51) * np.uint64(3)
lut = O.lut_from_table(2048, 16, [(m * 5 + 3) % 16 for m in range(16)], (1 << 63) // 16)
acc = eng.blind_rotate(cts[1:2], lut)
np.save("gpurun_out/f2k_dbg2.npy", acc)
os.makedirs("gpurun_out", exist_ok=True)
np.save("gpurun_out/f2k_dbg2.npy", acc)
print("ok")
