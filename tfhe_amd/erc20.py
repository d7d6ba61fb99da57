"""EncryptedERC20 on the GPU engine: the reference's flagship fhEVM contract flow on euint64 balances.

Restates tests/fhevm-suite/e2e/contracts/EncryptedERC20.sol operator for operator:
  mint(x)                 balances[owner] = FHE.add(balances[owner], x)                         :61-64
  transfer(to, amount)    canTransfer = FHE.le(amount, balances[from]); _transfer(...)           :87-95
  approve(spender, a)     allowances[owner][spender] = a                                         :120-126
  transferFrom(f, t, a)   _updateAllowance: allowed = le(a, allowance), can = le(a, balances[f]),
                          ok = and(can, allowed), allowance = select(ok, sub(allowance, a), allowance)
                                                                                                 :157-199
  _transfer(f, t, a, ok)  v = select(ok, a, 0); balances[t] = add(balances[t], v);
                          balances[f] = sub(balances[f], v)                                      :208-219
and is checked against the scenarios of tests/fhevm-suite/e2e/test/encryptedERC20/EncryptedERC20.ts
(mint 1000; transfer 1337 of 10000 -> 8663 / 1337; transfer 1337 of 1000 -> nothing moves;
transferFrom above the allowance -> nothing, at the allowance -> moves).

Two backends with the same operator semantics: "gate" (tfhe_amd.integer: 64 gate-bootstrapped bits,
P-GATE) and "radix" (tfhe_amd.radix: 32 blocks of 2 bits, P-FHEVM -- fhEVM's own encoding).  Every
operator of a transaction is one coroutine on the circuit; independent transactions can be stepped in
lockstep with ``Circuit.run_many`` (``transfer_ops``).
"""
from __future__ import annotations

from typing import Dict, Optional, Tuple


WIDTH = 64  # euint64 (EncryptedERC20.sol: mapping(address => euint64) balances)


class _Gate:
    def __init__(self, circuit):
        from . import integer as I
        self.I, self.c = I, circuit

    def encrypt(self, ck, v, seed=None, stream0=0):
        return self.I.FheUint.encrypt(self.c, ck, [v], WIDTH, seed=seed, stream0=stream0)

    def trivial(self, v):
        return self.I.FheUint.trivial(self.c, [v], WIDTH)

    def op(self, name, a, b=None):
        return self.I.fhevm_op(self.c, name, a, b)

    def and_(self, x, y):
        (r,) = yield [self.I.AND(x, y)]
        return r

    def select(self, cond, x, y):
        return self.I.FheUint(self.c, (yield from self.I.g_select(cond, x.bits, y.bits)))

    def decrypt(self, ck, v):
        return int(self.I.decrypt_bits(ck, v.bits)[0])


class _Radix:
    def __init__(self, circuit):
        from . import radix as R
        self.R, self.c = R, circuit

    def encrypt(self, ck, v, seed=None, stream0=0):
        return self.R.RadixUint.encrypt(self.c, ck, [v], WIDTH, seed=seed, stream0=stream0)

    def trivial(self, v):
        return self.R.RadixUint.trivial(self.c, [v], WIDTH)

    def op(self, name, a, b=None):
        return self.R.fhevm_op(self.c, name, a, b)

    def and_(self, x, y):
        (r,) = yield [(self.R._pack(x, y), self.R.T_AND1)]
        return r

    def select(self, cond, x, y):
        return self.R.RadixUint(self.c, (yield from self.R.g_select(self.c, cond, x.blocks, y.blocks)))

    def decrypt(self, ck, v):
        return int(v.decrypt(ck)[0])


class EncryptedERC20:
    """Encrypted balances and allowances of one token (EncryptedERC20.sol) on a Circuit of either layer."""

    def __init__(self, circuit, owner: str, backend: str = "gate"):
        self.b = _Gate(circuit) if backend == "gate" else _Radix(circuit)
        self.c = circuit
        self.owner = owner
        self.balances: Dict[str, object] = {}
        self.allowances: Dict[Tuple[str, str], object] = {}
        self.total_supply = 0

    def _bal(self, who: str):
        return self.balances.get(who) or self.b.trivial(0)

    # -- EncryptedERC20.sol:61-64 ------------------------------------------------------------------
    def mint(self, amount: int) -> None:
        self.balances[self.owner] = self.c.run(self.b.op("add", self._bal(self.owner), int(amount)))
        self.total_supply += int(amount)

    # -- :87-95 + _transfer :208-219 ---------------------------------------------------------------
    def transfer_op(self, sender: str, to: str, amount):
        """Coroutine: returns (new balance of sender, new balance of to)."""
        can = yield from self.b.op("le", amount, self._bal(sender))
        return (yield from self._move(sender, to, amount, can))

    def _move(self, frm: str, to: str, amount, ok):
        """_transfer (:208-219): balances[to] is written first and balances[from] is then computed from the
        stored value, so a self-transfer (frm == to) leaves the balance unchanged.  Callers store new_to
        first and new_from last, the contract's write order."""
        value = yield from self.b.select(ok, amount, self.b.trivial(0))
        new_to = yield from self.b.op("add", self._bal(to), value)
        from_bal = new_to if frm == to else self._bal(frm)
        new_from = yield from self.b.op("sub", from_bal, value)
        return new_from, new_to

    def transfer(self, sender: str, to: str, amount) -> None:
        new_from, new_to = self.c.run(self.transfer_op(sender, to, amount))
        self.balances[to] = new_to
        self.balances[sender] = new_from

    # -- :120-126 ----------------------------------------------------------------------------------
    def approve(self, owner: str, spender: str, amount) -> None:
        self.allowances[(owner, spender)] = amount

    # -- :157-163 + _updateAllowance :191-199 ------------------------------------------------------
    def transfer_from_op(self, spender: str, frm: str, to: str, amount):
        allowance = self.allowances.get((frm, spender)) or self.b.trivial(0)
        allowed = yield from self.b.op("le", amount, allowance)
        can = yield from self.b.op("le", amount, self._bal(frm))
        ok = yield from self.b.and_(can, allowed)
        left = yield from self.b.op("sub", allowance, amount)
        new_allowance = yield from self.b.select(ok, left, allowance)
        new_from, new_to = yield from self._move(frm, to, amount, ok)
        return new_allowance, new_from, new_to

    def transfer_from(self, spender: str, frm: str, to: str, amount) -> None:
        a, f, t = self.c.run(self.transfer_from_op(spender, frm, to, amount))
        self.allowances[(frm, spender)] = a
        self.balances[to] = t
        self.balances[frm] = f

    def balance_of(self, ck, who: str) -> int:
        return self.b.decrypt(ck, self._bal(who))

    def allowance(self, ck, owner: str, spender: str) -> int:
        a = self.allowances.get((owner, spender))
        return 0 if a is None else self.b.decrypt(ck, a)

    def encrypt_amount(self, ck, v: int, seed: Optional[int] = None, stream0: int = 0):
        """input.add64(v) (EncryptedERC20.ts:73): an encrypted euint64 transfer amount."""
        return self.b.encrypt(ck, v, seed=seed, stream0=stream0)


def transfer_ops(token: EncryptedERC20, transfers):
    """Independent transfers (distinct sender / recipient pairs) as coroutines for Circuit.run_many:
    all of them advance one circuit level per launch."""
    return [token.transfer_op(s, t, a) for s, t, a in transfers]
