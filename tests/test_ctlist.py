"""tfhe-rs compact ciphertext list ingest (tfhe_amd/ctlist.py) on CPU.

Pinned against the reference's own files, read in place (the test skips where /root/reference is absent):
  * the four ProvenCompactCiphertextList fixtures -- sdk/relayer/src/test/v1/ciphertext.ts:1 and
    src/test/assets/input-proof-payload-{1,2,3}.json `ciphertextWithInputVerification` -- parse to LWE
    compact lists whose DataKinds equal each payload's declared fheTypeEncryptionBitwidths and whose
    ciphertext counts equal ceil(blocks / 2) (packed: two 2-bit blocks per LWE);
  * the expansion convention: a compact list encrypted with the reference's real CompactPublicKey
    (src/test/keys/publicKey.bin) expands to LWEs that decrypt, under the compact-PKE secret key ingested
    from the paired ClientKey (privateKey.bin), to the packed values with noise far below Delta -- and a
    wrong convention does not.
The fixtures' own ciphertexts were encrypted under another network's key (they do not decrypt under
privateKey.bin with any convention), so their bits are parsed, not decrypted.
"""
import json
import os
import re

import numpy as np
import pytest

from tfhe_amd import ctlist, keyio

REF = "/root/reference/sdk/relayer/src/test"
pytestmark = pytest.mark.skipif(not os.path.isdir(REF), reason="reference fixtures not present")


def _fixtures():
    out = []
    t = open(os.path.join(REF, "v1", "ciphertext.ts")).read()
    out.append(("v1/ciphertext.ts", bytes.fromhex(re.findall(r"'([0-9a-f]+)'", t)[0]), [32], None))
    for i in (1, 2, 3):
        d = json.load(open(os.path.join(REF, "assets", f"input-proof-payload-{i}.json")))
        h = d["ciphertextWithInputVerification"]
        out.append((f"input-proof-payload-{i}.json", bytes.fromhex(h[2:] if h.startswith("0x") else h),
                    d["fheTypeEncryptionBitwidths"], d.get("values")))
    return out


def _blocks_of(bits):
    return 1 if bits == 2 else bits // 2          # ebool travels as one block (bitwidth 2 in fhEVM)


def test_reference_lists_parse_and_match_declared_types():
    for name, data, widths, _ in _fixtures():
        cl = ctlist.load_compact_list(data)
        assert cl.lwe_dim == 2048 and cl.message_modulus == 4 and cl.carry_modulus == 4, name
        assert [n for _, n in cl.kinds] == [_blocks_of(w) for w in widths], (name, cl.kinds, widths)
        assert [k for k, _ in cl.kinds] == [ctlist.KIND_BOOLEAN if w == 2 else ctlist.KIND_UNSIGNED for w in widths]
        assert cl.count == -(-cl.blocks // 2), name            # packed: two blocks per LWE
        assert cl.masks.shape == (1, 2048) and cl.bodies.shape == (cl.count,)
        ex = ctlist.expand(cl)
        assert ex.shape == (cl.count, 2049)


def test_expansion_convention_against_reference_key_pair():
    tk = keyio.load_client_key(os.path.join(REF, "keys", "privateKey.bin"))
    cpk = keyio.load_compact_public_key(os.path.join(REF, "keys", "publicKey.bin"))
    s = tk.pke_key.astype(np.uint64)
    vals = [1, 255, 0xFFFFFFFF, 0xFFFFFFFFFFFFFFFF]          # the clear values of input-proof-payload-2.json
    kinds = [(ctlist.KIND_BOOLEAN, 1), (0, 4), (0, 16), (0, 32)]
    packed = ctlist.pack_blocks(ctlist.value_blocks(vals, kinds))
    assert len(packed) == 27
    cl = ctlist.encrypt_compact(cpk, packed, kinds, np.random.default_rng(2))
    ex = ctlist.expand(cl)
    D = ctlist.DELTA_PACKED
    with np.errstate(over="ignore"):
        ph = ex[:, -1] - (ex[:, :-1] * s[None, :]).sum(axis=1)
    err = [((int(p) - v * D + (1 << 63)) % (1 << 64)) - (1 << 63) for p, v in zip(ph, packed)]
    assert max(abs(e) for e in err) < (1 << 32)              # TUniform(17) noise x a 2048-term binary sum
    blocks = [b for v in packed for b in (v % 4, v // 4)][:cl.blocks]
    assert ctlist.unpack_values(blocks, kinds) == vals
    # negative control: reading the masks in the plain convolution order does not decrypt
    with np.errstate(over="ignore"):
        wrong = cl.bodies - keyio.negacyclic_mul_binary(cl.masks[0], s)[:cl.count]
    assert max(abs(((int(p) - v * D + (1 << 63)) % (1 << 64)) - (1 << 63)) for p, v in zip(wrong, packed)) > (1 << 50)
