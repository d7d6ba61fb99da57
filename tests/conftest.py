"""Shared fixtures.  `-m gpu` tests need an MI355X; everything else runs on CPU."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

KEY_SEED = 0x7F4E0001  # SURVEY §8d synthetic-input key seed


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libtfhe_hip.so on the device)")
    config.addinivalue_line("markers", "slow: long CPU-oracle cross-check")


@pytest.fixture(scope="session")
def oracle_mod():
    from oracle import oracle as O
    O.lib()
    return O


@pytest.fixture(scope="session")
def gate_params(oracle_mod):
    return oracle_mod.params(0)


@pytest.fixture(scope="session")
def oracle_keys(oracle_mod, gate_params):
    """P-GATE keys from the oracle (same ChaCha20 streams as the product keygen)."""
    return oracle_mod.Keys(gate_params, KEY_SEED)


@pytest.fixture(scope="session")
def product_keys():
    import tfhe_amd
    return tfhe_amd.gen_keys(tfhe_amd.Params.preset(tfhe_amd.PRESET_GATE), KEY_SEED)


@pytest.fixture(scope="session")
def engine(product_keys):
    import tfhe_amd
    ck, sk = product_keys
    eng = tfhe_amd.Engine(ck.params, 0)
    eng.load_keys(sk)
    yield eng
    eng.close()


def load_golden(name):
    path = os.path.join(ROOT, "tests", "golden", name)
    with np.load(path, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


# ---- P-FHEVM (N=2048, KS->PBS) fixtures shared by the gpu tests --------------------------------
@pytest.fixture(scope="session")
def fhevm_keys():
    import tfhe_amd
    return tfhe_amd.gen_keys(tfhe_amd.Params.preset(tfhe_amd.PRESET_FHEVM), KEY_SEED)


@pytest.fixture(scope="session")
def fhevm_engine(fhevm_keys):
    import tfhe_amd
    ck, sk = fhevm_keys
    eng = tfhe_amd.Engine(ck.params, 0)
    eng.load_keys(sk)
    yield eng
    eng.close()


# ---- FFT64 engines (tfhe-rs's f64-FFT arithmetic) for message-level suites -------------------
@pytest.fixture(scope="session")
def gate_fft_keys():
    import tfhe_amd
    return tfhe_amd.gen_keys(tfhe_amd.Params.preset(tfhe_amd.PRESET_GATE_FFT), KEY_SEED)


@pytest.fixture(scope="session")
def gate_fft_engine(gate_fft_keys):
    import tfhe_amd
    ck, sk = gate_fft_keys
    eng = tfhe_amd.Engine(ck.params, 0)
    eng.load_keys(sk)
    yield eng
    eng.close()


@pytest.fixture(scope="session")
def fhevm_fft_keys():
    import tfhe_amd
    return tfhe_amd.gen_keys(tfhe_amd.Params.preset(tfhe_amd.PRESET_FHEVM_FFT), KEY_SEED)


@pytest.fixture(scope="session")
def fhevm_fft_engine(fhevm_fft_keys):
    import tfhe_amd
    ck, sk = fhevm_fft_keys
    eng = tfhe_amd.Engine(ck.params, 0)
    eng.load_keys(sk)
    yield eng
    eng.close()


# ---- fhEVM operator KATs (tests/golden/fhevm_kats.json: clear values stored as decimal strings) ----------
KATS_PATH = os.path.join(ROOT, "tests", "golden", "fhevm_kats.json")


def load_kats(max_width: int = 256):
    """The reference's 2,394 fhEVM KATs with args / expect as Python ints; max_width drops overloads
    wider than that (operand or result type)."""
    import json

    def width(t):
        return 1 if t == "ebool" else int(t.lstrip("e").replace("uint", ""))

    with open(KATS_PATH) as f:
        kats = json.load(f)
    out = []
    for k in kats:
        if max(width(t) for t in k["types"] + [k["result_type"]]) > max_width:
            continue
        out.append(dict(k, args=[int(a) for a in k["args"]], expect=int(k["expect"])))
    return out
