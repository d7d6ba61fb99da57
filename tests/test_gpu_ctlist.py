"""Compact-list ingest into the GPU engine (tfhe_amd/ctlist.py): an fhEVM client input --
one packed compact list under a CompactPublicKey, in the format of the reference's
ProvenCompactCiphertextList fixtures -- is expanded, cast by a P-FHEVM engine whose keyswitch key is the
casting key (compact-PKE key -> small key) into radix blocks under the computation key (one unpacking PBS
per block), and then used by fhEVM operators on the regular engine.  The compact-PKE key here is generated
fresh (the reference's key pair is secret-key material that stays out of this repository; its conventions
are pinned on CPU by tests/test_ctlist.py)."""
import numpy as np
import pytest

import tfhe_amd
from tfhe_amd import ctlist
from tfhe_amd import radix as R

pytestmark = pytest.mark.gpu


def test_compact_list_cast_and_compute(fhevm_fft_engine, fhevm_fft_keys):
    ck, _ = fhevm_fft_keys
    rng = np.random.default_rng(0xC0)
    pke_key = rng.integers(0, 2, 2048).astype(np.uint64)
    cpk = ctlist.gen_compact_public_key(pke_key, rng)
    vals = [1, 255, 0xFFFFFFFF, 0xFFFFFFFFFFFFFFFF, 12345678901234567890]   # payload-2's inputs + one euint64
    kinds = [(ctlist.KIND_BOOLEAN, 1), (0, 4), (0, 16), (0, 32), (0, 32)]
    cl = ctlist.encrypt_compact(cpk, ctlist.pack_blocks(ctlist.value_blocks(vals, kinds)), kinds, rng)
    ex = ctlist.expand(cl)
    with tfhe_amd.Engine(ck.params, 0) as cast:
        cast.load_keys(ctlist.casting_keys(ck, pke_key, seed=0x5EED))
        blocks = ctlist.cast_to_blocks(cast, ex, cl.blocks)
    assert blocks.shape == (cl.blocks, 2049)
    got = ck.decrypt(blocks, R.SPACE)
    assert ctlist.unpack_values(got, kinds) == vals
    # the cast blocks are ordinary radix operands: euint64 a + b and a < b on the computation engine
    c = R.RadixCircuit(fhevm_fft_engine)
    a = R.RadixUint(c, blocks[21:53][None])
    b = R.RadixUint(c, blocks[53:85][None])
    s, lt = c.run_many([R.fhevm_op(c, "add", a, b), R.fhevm_op(c, "lt", a, b)])
    assert int(s.decrypt(ck)[0]) == (vals[3] + vals[4]) % (1 << 64)
    assert int(ck.decrypt(lt, R.SPACE)[0]) == int(vals[3] < vals[4])
