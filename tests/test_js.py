"""The N-API boundary: js/ (addon + JS shim) driven by node.  CPU checks run here; the GPU checks
are marked gpu.  Key material through N-API must equal the Python/ctypes path byte-for-byte."""
import hashlib
import json
import os
import shutil
import subprocess

import numpy as np
import pytest

from conftest import ROOT

NODE = shutil.which("node")
ADDON = os.path.join(ROOT, "js", "build", "tfhe_napi.node")
pytestmark = pytest.mark.skipif(NODE is None or not os.path.exists("/usr/include/node/node_api.h"),
                                reason="node / N-API headers not available")


def _ensure_addon():
    if not os.path.exists(ADDON):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "js")], check=True)


def _run(script, timeout, *args):
    _ensure_addon()
    r = subprocess.run([NODE, os.path.join(ROOT, "tests", "js", script), *args], capture_output=True, text=True,
                       timeout=timeout, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_js_addon_cpu(product_keys):
    out = _run("cpu_check.js", 300)
    assert out["exports"] == sorted(["paramsPreset", "keygen", "encrypt", "phase", "lutConstant", "lutFromTable",
                                     "createEngine", "destroyEngine", "loadKeys", "pbs", "nand", "lastError",
                                     "keyswitch", "blindRotate", "engineInfo", "createPacker", "createSquasher",
                                     "destroyAux", "pksKeygen", "snsKeygen", "loadAuxKey", "packCompress", "squash",
                                     "extractGlwe", "glwePhase", "snsPhase"])
    ck, sk = product_keys
    sha = lambda a: hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()
    assert out["lwe_key_sha"] == sha(ck.lwe_key)
    assert out["bsk_sha"] == sha(sk.bsk)
    assert out["ksk_sha"] == sha(sk.ksk)
    cts = ck.encrypt_bool(np.array([True, False, True]), seed=0xC0FFEE02, stream0=5)
    assert out["ct_sha"] == sha(cts)
    assert out["err"] == "-1"
    # no public default seed -- keys and encryptions from OS entropy, fixed seeds only with dev
    assert out["entropy_keys_differ"] and out["entropy_cts_differ"]
    assert out["seed_refused"] and out["seed_dev_ok"]
    assert out["default_params"] == 1  # LuxFHELocalClient defaults to the FFT64 engine
    assert out["unseal_sync"] is True  # a bigint, not a Promise (luxfhejs index.ts:146)
    if out["engine"] != "created":  # no GPU here: a clean error, not an abort
        assert out["engine"] in ("-1", "-3")


@pytest.mark.gpu
@pytest.mark.parametrize("preset", ["0", "2"])  # P-GATE on the NTT and on the FFT64 engine
def test_js_addon_gpu(preset):
    assert _run("gpu_check.js", 600, preset)["ok"] is True


def _run_plain(script, *args, timeout=600):
    _ensure_addon()
    r = subprocess.run([NODE, os.path.join(ROOT, "tests", "js", script), *args], capture_output=True, text=True,
                       timeout=timeout, cwd=ROOT)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    return r.stdout.strip().splitlines()[-1]


def test_js_integer_kats_cpu():
    """js/integer.js replays all 2,394 fhEVM KATs (ebool .. euint256; cleartext test double) with the same
    launch and PBS counts as tfhe_amd/integer.py (the block carry-out circuit's cost model included)."""
    import sys
    sys.path.insert(0, os.path.dirname(__file__))
    from conftest import load_kats
    from test_integer import CleartextEngine, build_kat_op
    from tfhe_amd import integer as I
    kats = load_kats()
    c = I.Circuit(CleartextEngine(n=1))
    c.run_many([build_kat_op(c, k) for k in kats])
    assert _run_plain("integer_check.js") == f"OK 2394 KATs, {c.launches} launches, {c.pbs_count} PBS"


def test_js_radix_kats_cpu():
    """js/radix.js replays all 2,394 radix-layer fhEVM KATs (ebool .. euint256) with the same launch and PBS counts as
    tfhe_amd/radix.py (tests/test_radix.py) — the two layers build identical circuits."""
    import sys
    sys.path.insert(0, os.path.dirname(__file__))
    from conftest import load_kats
    from test_radix import CleartextRadixCircuit, kat_op, supported
    kats = [k for k in load_kats() if supported(k)]
    c = CleartextRadixCircuit(N=16)
    c.run_many([kat_op(c, k) for k in kats])
    assert _run_plain("radix_check.js") == f"OK {len(kats)} {c.launches} {c.pbs_count}"


def test_js_server_cpu():
    """js/server.js over HTTP with the reference's request shapes (fhe.test.ts, hardhat plugin)."""
    assert _run_plain("server_check.js").startswith("OK server")


def test_js_server_fhevm_cpu():
    """The same requests on P-FHEVM radix blocks (server --params fhevm)."""
    assert _run_plain("server_check.js", "fhevm").startswith("OK server (cpu double, fhevm radix)")


@pytest.mark.gpu
def test_js_server_fhevm_gpu():
    assert _run_plain("server_check.js", "fhevm-gpu", timeout=900).startswith("OK server (gpu, fhevm radix)")


@pytest.mark.gpu
def test_js_server_gpu():
    assert _run_plain("server_check.js", "gpu", timeout=900).startswith("OK server (gpu)")


@pytest.mark.gpu
def test_js_adjacent_gpu(tmp_path):
    """packCompress and squash through N-API (compression.rs:222,276; the sns-worker,
    coprocessor-docker-compose.yml:124-140) equal the Python / ctypes path byte for byte on the same keys."""
    import tfhe_amd
    from conftest import KEY_SEED
    from tfhe_amd import compression as C
    from tfhe_amd import sns as S
    pp = C.PksParams.preset(C.PKS_PRESET_ML2048)
    in_key = np.random.default_rng(5).integers(0, 2, pp.in_dim).astype(np.uint64)
    count = 2048 + 77                                         # one full group + a ragged one
    lwes = np.random.default_rng(6).integers(0, 2 ** 64 - 1, size=(count, pp.in_dim + 1), dtype=np.uint64)
    in_key.tofile(tmp_path / "in_key.bin")
    lwes.tofile(tmp_path / "lwes.bin")
    out = _run("adjacent_gpu_check.js", 600, str(tmp_path), str(KEY_SEED))
    assert out["ok"] and out["squash_decrypt_ok"] and out["groups"] == 2
    # 26-bit storage: each coefficient moves by < 2^37, the phase by < 2^44 over 2048 key bits (the bound
    # tests/test_gpu_compression.py decodes messages spaced 2^45 apart under)
    assert out["extract_max_err_log2"] <= 44
    ck_pks = C.CompressionKey(pp, KEY_SEED, in_key)
    assert np.array_equal(np.fromfile(tmp_path / "js_out_key.bin", dtype=np.uint64), ck_pks.post_packing_key)
    packer = C.Packer(pp, 0).load_key(ck_pks)
    glwes = packer.pack(lwes)
    comp = packer.compress_ciphertexts_into_list(lwes)
    packer.close()
    assert np.array_equal(np.fromfile(tmp_path / "js_glwes.bin", dtype=np.uint64), glwes.reshape(-1))
    assert np.array_equal(np.fromfile(tmp_path / "js_packed.bin", dtype=np.uint64),
                          np.concatenate([c.packed for c in comp]))
    params = tfhe_amd.Params.preset(tfhe_amd.PRESET_FHEVM_FFT)
    ck, sk = tfhe_amd.gen_keys(params, KEY_SEED)
    msgs = np.array([(i * 7 + 3) % 16 for i in range(64)], dtype=np.uint64)
    cts = ck.encrypt(msgs, 16, seed=KEY_SEED + 1)
    sp = S.SnsParams.preset(0)
    key = S.SquashedKey(sp, KEY_SEED, ck.lwe_key)
    with tfhe_amd.Engine(params, 0) as eng:
        eng.load_keys(sk)
        sq = S.Squasher(sp, 0).load_key(key)
        ref = S.squash_noise(eng, sq, cts)
        sq.close()
    assert np.array_equal(np.fromfile(tmp_path / "js_squash.bin", dtype=np.uint64), ref.reshape(-1))
