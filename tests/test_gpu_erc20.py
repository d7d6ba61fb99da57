"""EncryptedERC20 on the MI355X (tfhe_amd/erc20.py): the reference's euint64 token scenarios
(tests/fhevm-suite/e2e/test/encryptedERC20/EncryptedERC20.ts:41,73: mint, transfer of input.add64(1337),
a refused transfer, transferFrom above / at the allowance) with real encryptions, on the boolean layer
(P-GATE FFT64 engine) and on fhEVM's radix blocks (P-FHEVM FFT64 engine)."""
import pytest

from tfhe_amd import integer as I
from tfhe_amd import radix as R
from tfhe_amd.erc20 import EncryptedERC20

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("backend", ["gate", "radix"])
def test_erc20_scenarios_gpu(request, backend):
    eng = request.getfixturevalue("gate_fft_engine" if backend == "gate" else "fhevm_fft_engine")
    ck, _ = request.getfixturevalue("gate_fft_keys" if backend == "gate" else "fhevm_fft_keys")

    def token():
        c = I.Circuit(eng) if backend == "gate" else R.RadixCircuit(eng)
        return EncryptedERC20(c, "alice", backend)

    amt = lambda tok, v: tok.encrypt_amount(ck, v)   # input.add64(v): fresh entropy per encryption
    tok = token()
    tok.mint(1000)
    assert tok.balance_of(ck, "alice") == 1000
    tok.mint(9000)
    tok.transfer("alice", "bob", amt(tok, 1337))
    assert tok.balance_of(ck, "alice") == 8663 and tok.balance_of(ck, "bob") == 1337
    tok2 = token()
    tok2.mint(1000)
    tok2.transfer("alice", "bob", amt(tok2, 1337))
    assert tok2.balance_of(ck, "alice") == 1000 and tok2.balance_of(ck, "bob") == 0
    tok3 = token()
    tok3.mint(10000)
    tok3.approve("alice", "bob", amt(tok3, 1337))
    tok3.transfer_from("bob", "alice", "bob", amt(tok3, 1338))
    assert tok3.balance_of(ck, "alice") == 10000 and tok3.balance_of(ck, "bob") == 0
    tok3.transfer_from("bob", "alice", "bob", amt(tok3, 1337))
    assert tok3.balance_of(ck, "alice") == 8663 and tok3.balance_of(ck, "bob") == 1337
    assert tok3.allowance(ck, "alice", "bob") == 0
