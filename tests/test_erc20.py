"""EncryptedERC20 (tfhe_amd/erc20.py) on CPU with the cleartext test doubles of both integer layers:
the reference's scenarios (tests/fhevm-suite/e2e/test/encryptedERC20/EncryptedERC20.ts) on euint64
balances.  The MI355X run with real encryptions is tests/test_gpu_erc20.py."""
import pytest

from tfhe_amd import integer as I
from tfhe_amd.erc20 import EncryptedERC20, transfer_ops
from test_integer import CleartextEngine, ClearKey
from test_radix import CleartextRadixCircuit
from test_radix import ClearKey as RadixClearKey


def _token(backend):
    if backend == "gate":
        return EncryptedERC20(I.Circuit(CleartextEngine(n=1)), "alice", "gate"), ClearKey()
    return EncryptedERC20(CleartextRadixCircuit(N=16), "alice", "radix"), RadixClearKey()


def _amount(tok, v):
    return tok.b.trivial(v)   # the doubles take trivial ciphertexts (input.add64(v) on the GPU)


@pytest.mark.parametrize("backend", ["gate", "radix"])
def test_erc20_reference_scenarios(backend):
    tok, ck = _token(backend)
    tok.mint(1000)                                                # "should mint the contract"
    assert tok.balance_of(ck, "alice") == 1000 and tok.total_supply == 1000
    tok.mint(9000)
    tok.transfer("alice", "bob", _amount(tok, 1337))              # "should transfer tokens between two users"
    assert tok.balance_of(ck, "alice") == 10000 - 1337 and tok.balance_of(ck, "bob") == 1337
    tok2, ck2 = _token(backend)                                   # "should not transfer tokens between two users"
    tok2.mint(1000)
    tok2.transfer("alice", "bob", _amount(tok2, 1337))
    assert tok2.balance_of(ck2, "alice") == 1000 and tok2.balance_of(ck2, "bob") == 0
    tok3, ck3 = _token(backend)                                   # "transferFrom only if allowance is sufficient"
    tok3.mint(10000)
    tok3.approve("alice", "bob", _amount(tok3, 1337))
    tok3.transfer_from("bob", "alice", "bob", _amount(tok3, 1338))
    assert tok3.balance_of(ck3, "alice") == 10000 and tok3.balance_of(ck3, "bob") == 0
    assert tok3.allowance(ck3, "alice", "bob") == 1337
    tok3.transfer_from("bob", "alice", "bob", _amount(tok3, 1337))
    assert tok3.balance_of(ck3, "alice") == 10000 - 1337 and tok3.balance_of(ck3, "bob") == 1337
    assert tok3.allowance(ck3, "alice", "bob") == 0


@pytest.mark.parametrize("backend", ["gate", "radix"])
def test_erc20_lockstep_transfers(backend):
    """Independent transfers advance together (one launch per circuit level for all of them)."""
    tok, ck = _token(backend)
    tok.mint(1 << 40)
    users = [f"u{i}" for i in range(8)]
    for u in users:
        tok.transfer("alice", u, _amount(tok, 1000))
    launches0 = tok.c.launches
    outs = tok.c.run_many(transfer_ops(tok, [(users[i], users[i + 4], _amount(tok, 100 * (i + 1))) for i in range(4)]))
    depth = tok.c.launches - launches0
    for i, (nf, nt) in enumerate(outs):
        tok.balances[users[i]], tok.balances[users[i + 4]] = nf, nt
    for i in range(4):
        assert tok.balance_of(ck, users[i]) == 1000 - 100 * (i + 1)
        assert tok.balance_of(ck, users[i + 4]) == 1000 + 100 * (i + 1)
    single0 = tok.c.launches
    tok.transfer(users[0], users[1], _amount(tok, 1))
    assert depth == tok.c.launches - single0       # four transfers cost the launches of one


@pytest.mark.parametrize("backend", ["gate", "radix"])
def test_erc20_self_transfer_keeps_balance(backend):
    """EncryptedERC20.sol:211-216 writes balances[to] first and computes balances[from] from the stored
    value: a transfer (or transferFrom) to oneself moves nothing and creates no tokens."""
    tok, ck = _token(backend)
    tok.mint(5000)
    tok.transfer("alice", "alice", _amount(tok, 1200))
    assert tok.balance_of(ck, "alice") == 5000
    tok.approve("alice", "bob", _amount(tok, 700))
    tok.transfer_from("bob", "alice", "alice", _amount(tok, 700))
    assert tok.balance_of(ck, "alice") == 5000
    assert tok.allowance(ck, "alice", "bob") == 0
