"""Packing keyswitch on the MI355X (tfhe_amd/csrc/pks.hip) against the oracle: bit-exact GLWEs for
partial groups, the full 2048-LWE group and several groups in one call checked by decryption, and the
compress -> extract round trip (ml/extensions/rust/src/compression.rs:246-291 shape)."""
import numpy as np
import pytest

from tfhe_amd import compression as C
from test_compression import SEED, encrypt_lwes

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def setup(oracle_mod):
    pp = C.PksParams.preset(C.PKS_PRESET_ML2048)
    opp = oracle_mod.pks_params(0)
    in_key = np.random.default_rng(5).integers(0, 2, pp.in_dim).astype(np.uint64)
    ck = C.CompressionKey(pp, SEED, in_key)
    ok = oracle_mod.PksKeys(opp, SEED, in_key)
    packer = C.Packer(pp, 0).load_key(ck)
    yield pp, opp, ck, ok, packer
    packer.close()


@pytest.mark.parametrize("count", [1, 7, 65])
def test_pack_vs_oracle(setup, oracle_mod, count):
    pp, opp, ck, ok, packer = setup
    rng = np.random.default_rng(count)
    lwes = rng.integers(0, 2 ** 64 - 1, size=(count, pp.in_dim + 1), dtype=np.uint64)
    g = packer.pack(lwes)
    assert g.shape == (1, pp.glwe_len)
    assert np.array_equal(g[0], oracle_mod.pks_pack(opp, ok, lwes))


def test_pack_many_groups_decrypt(setup, oracle_mod):
    """2 full groups + a partial one in one call (chunked GEMM workspaces); last group bit-exact
    with the oracle, every coefficient of every group decrypts to its message."""
    pp, opp, ck, ok, packer = setup
    count = 2 * 2048 + 9
    msgs = (np.arange(count, dtype=np.uint64) % 4096) << np.uint64(44)
    lwes = encrypt_lwes(oracle_mod, ok.in_key, msgs, seed=11)
    g = packer.pack(lwes)
    assert g.shape == (3, pp.glwe_len)
    assert np.array_equal(g[2], oracle_mod.pks_pack(opp, ok, lwes[4096:]))
    for grp in range(3):
        ph = C.glwe_phase(1, 2048, ck.post_packing_key, g[grp])
        n = min(2048, count - grp * 2048)
        err = (ph[:n] - msgs[grp * 2048: grp * 2048 + n]).view(np.int64)
        assert np.abs(err).max() < 2 ** 43, grp


def test_compress_ciphertexts_into_list(setup, oracle_mod):
    pp, opp, ck, ok, packer = setup
    count = 3000
    msgs = (np.arange(count, dtype=np.uint64) * 7 % 2048) << np.uint64(45)
    lwes = encrypt_lwes(oracle_mod, ok.in_key, msgs, seed=12)
    comp = packer.compress_ciphertexts_into_list(lwes)
    assert [c.bodies for c in comp] == [2048, 952]
    raw = sum(lwes.nbytes for _ in [0])
    assert sum(c.nbytes for c in comp) * 10 < raw            # 2049 u64 per LWE -> ~ 1 coefficient each
    got = []
    for c in comp:
        ph = C.glwe_phase(1, 2048, ck.post_packing_key, c.extract())[:c.bodies]
        got.append(((ph + np.uint64(1 << 44)) >> np.uint64(45)) % np.uint64(2048))
    assert np.array_equal(np.concatenate(got), (np.arange(count, dtype=np.uint64) * 7) % 2048)


def test_pack_async_orders_with_torch_default_stream(setup):
    import torch
    pp, opp, ck, ok, packer = setup
    lwes = np.random.default_rng(3).integers(0, 2 ** 64 - 1, size=(40, pp.in_dim + 1), dtype=np.uint64)
    ref = packer.pack(lwes)
    dev = torch.device("cuda", 0)
    d_in = torch.from_numpy(lwes.view(np.int64)).to(dev)
    d_out = torch.zeros((1, pp.glwe_len), dtype=torch.int64, device=dev)
    packer.pack_async(d_in, 40, d_out)            # torch's current (default) stream
    assert np.array_equal(d_out.cpu().numpy().view(np.uint64), ref)
