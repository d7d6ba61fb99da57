"""tfhe-rs key ingest (tfhe_amd/keyio.py) against the reference's own key fixtures.

The fixtures (sdk/relayer/src/test/keys/{privateKey,publicKey}.bin) are read IN PLACE from
/root/reference (they are not copied into this repository); the tests skip where it is absent
(the GPU box).  Pins:
  * the parameter block decodes to SURVEY App. A's P-FHEVM values;
  * the compact public key is an encryption of zero under the ingested PKE secret key
    (|body - mask (*) reverse(s)| <= 2^17 = the TUniform(17) bound) — real tfhe-rs output;
  * the engine's server keys for the ingested secret keys equal the oracle's (same streams), and
    host encryption/decryption round-trips under the fhEVM key.
"""
import os

import numpy as np
import pytest

import tfhe_amd
from tfhe_amd import keyio

KEYS = "/root/reference/sdk/relayer/src/test/keys"
pytestmark = pytest.mark.skipif(not os.path.exists(os.path.join(KEYS, "privateKey.bin")),
                                reason="reference key fixtures not present (read in place, never copied)")


@pytest.fixture(scope="module")
def tk():
    return keyio.load_client_key(os.path.join(KEYS, "privateKey.bin"))


def test_client_key_params_and_keys(tk):
    P = tk.params
    assert (P["lwe_dimension"], P["glwe_dimension"], P["polynomial_size"]) == (918, 1, 2048)
    assert (P["pbs_base_log"], P["pbs_level"], P["ks_base_log"], P["ks_level"]) == (23, 1, 4, 4)
    assert (P["message_modulus"], P["carry_modulus"], P["max_noise_level"]) == (4, 4, 5)
    assert P["lwe_noise"] == "TUniform(45)" and P["glwe_noise"] == "TUniform(17)"
    assert abs(P["log2_p_fail"] + 129.15284804376165) < 1e-12
    assert P["ms_noise_reduction_zeros"] == 1449 and P["ms_bound"] == 2.0 ** 58
    assert tk.glwe_key.shape == (2048,) and int(tk.glwe_key.sum()) == 996
    assert tk.lwe_key.shape == (918,) and int(tk.lwe_key.sum()) == 460
    assert tk.pke_key.shape == (2048,) and int(tk.pke_key.sum()) == 975
    assert tk.pke_params == {"lwe_dimension": 2048, "noise_bound_log2": 17}


def test_compact_public_key_is_encryption_of_zero(tk):
    mask, body = keyio.load_compact_public_key(os.path.join(KEYS, "publicKey.bin"))
    assert mask.shape == body.shape == (2048,)
    noise = keyio.compact_public_key_noise(mask, body, tk.pke_key)
    assert noise <= 2 ** tk.pke_params["noise_bound_log2"]
    wrong = tk.pke_key.copy()
    wrong[5] ^= np.uint64(1)
    assert keyio.compact_public_key_noise(mask, body, wrong) > 2 ** 60


def test_engine_keys_from_ingested_client_key(tk, oracle_mod):
    ck, sk = keyio.to_engine_keys(tk, seed=0x5EED)
    ok = oracle_mod.Keys.from_secret(oracle_mod.params(1), 0x5EED, tk.lwe_key, tk.glwe_key)
    assert np.array_equal(sk.bsk, ok.bsk) and np.array_equal(sk.ksk, ok.ksk)
    msgs = np.arange(16, dtype=np.uint64)
    cts = ck.encrypt(msgs, 16, seed=3)
    assert cts.shape == (16, 2049)
    assert np.array_equal(ck.decrypt(cts, 16), msgs)
    # the ciphertexts are LWE under the fhEVM GLWE key read from the file
    assert np.array_equal(ck.glwe_key, tk.glwe_key)


def test_malformed_inputs_refused():
    data = open(os.path.join(KEYS, "privateKey.bin"), "rb").read()
    with pytest.raises(keyio.KeyFormatError):
        keyio.load_client_key(data[:4000])
    with pytest.raises(keyio.KeyFormatError):
        keyio.load_client_key(open(os.path.join(KEYS, "publicKey.bin"), "rb").read())
    bad = bytearray(data)
    bad[8:11] = b"9.9"
    with pytest.raises(keyio.KeyFormatError):
        keyio.load_client_key(bytes(bad))
    p = tfhe_amd.Params.preset(tfhe_amd.PRESET_FHEVM)
    ck = tfhe_amd.ClientKey(p, 0, np.full(918, 2, dtype=np.uint64), np.zeros(2048, dtype=np.uint64))
    with pytest.raises(tfhe_amd.TfheError):
        tfhe_amd.server_keygen(ck)
