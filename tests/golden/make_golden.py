"""Generate the committed golden fixtures from the CPU oracle (run from the repo root):

    python tests/golden/make_golden.py

Fixtures are DATA (inputs + oracle outputs); keys are not stored, only their seed
(conftest.KEY_SEED): every consumer regenerates the P-GATE keys deterministically.
Ciphertext-level parity with tfhe-rs is "parity unpinned" (see oracle/tfhe_oracle.h):
these vectors pin the GPU path to the oracle, not to the reference's absent core.
"""
import hashlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402

KEY_SEED = 0x7F4E0001
OUT = os.path.dirname(os.path.abspath(__file__))


def main():
    P = O.P
    rng = np.random.default_rng(20261015)
    # 1. NTT vectors (N=1024): natural-order negacyclic NTT mod p
    polys = rng.integers(0, P, size=(4, 1024), dtype=np.uint64)
    polys[0] = 0
    polys[0, 0] = 1                      # delta -> all ones
    polys[1] = 0
    polys[1, 1] = 1                      # X -> psi^(2j+1)
    np.savez(os.path.join(OUT, "ntt_1024.npz"), input=polys, output=O.ntt_fwd(polys), psi=np.uint64(O.psi(1024)))

    prm = O.params(0)
    keys = O.Keys(prm, KEY_SEED)
    # 2. full PBS (BR + SE + KS) of 8 ciphertexts with 3 LUTs
    msgs = np.array([O.encode_bit(b) for b in (1, 0, 1, 1, 0, 0, 1, 0)], dtype=np.uint64)
    cts = keys.encrypt(msgs, seed=0xC0FFEE01, stream0=0)
    luts = np.stack([
        O.lut_constant(1024, O.MU),
        O.lut_from_table(1024, 4, [0, 1, 2, 3], (1 << 63) // 4),
        O.lut_from_table(1024, 4, [3, 2, 1, 0], (1 << 63) // 4),
    ])
    lut_index = np.array([0, 1, 2, 0, 1, 2, 0, 1], dtype=np.uint32)
    out = O.pbs_batch(prm, keys, cts, luts, lut_index)
    # stage outputs for the first ciphertext
    acc = O.blind_rotate(prm, keys, cts[0], luts[0])
    big = O.sample_extract(prm, acc)
    np.savez(os.path.join(OUT, "pbs_gate.npz"), key_seed=np.uint64(KEY_SEED), lwe_in=cts, luts=luts,
             lut_index=lut_index, lwe_out=out, acc0=acc, big0=big, ks0=O.keyswitch(prm, keys, big))
    # 3. NAND truth table
    c = keys.encrypt([O.encode_bit(b) for b in (0, 0, 1, 1, 0, 1, 0, 1)], seed=0xC0FFEE02)
    c1, c2 = c[:4], c[4:]
    nand = np.stack([O.nand(prm, keys, c1[i], c2[i]) for i in range(4)])
    np.savez(os.path.join(OUT, "nand_gate.npz"), c1=c1, c2=c2, out=nand,
             expect=np.array([1, 1, 1, 0], dtype=np.uint8))
    # 4. 64-PBS batch digest (inputs regenerated from the seed by the test)
    msgs = np.array([O.encode_bit(int(b)) for b in rng.integers(0, 2, 64)], dtype=np.uint64)
    cts = keys.encrypt(msgs, seed=0xC0FFEE03, stream0=0)
    out = O.pbs_batch(prm, keys, cts, luts[:1])
    np.savez(os.path.join(OUT, "pbs_batch64.npz"), msgs=msgs, input_seed=np.uint64(0xC0FFEE03),
             sha256_in=np.frombuffer(hashlib.sha256(cts.tobytes()).digest(), dtype=np.uint8),
             sha256_out=np.frombuffer(hashlib.sha256(out.tobytes()).digest(), dtype=np.uint8))
    print("golden fixtures written to", OUT)


if __name__ == "__main__":
    main()
