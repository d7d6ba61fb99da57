"""Extract the fhEVM operator known-answer tests from the reference's test files into a JSON
fixture (DATA: operator, operand types, clear inputs, expected clear output).

Source (read as text, at generation time only):
  /root/reference/tests/fhevm-suite/e2e/test/fhevmOperations{1..13}.ts
Each test there encrypts clear inputs, runs one Solidity FHE operator and asserts the decrypted
result (e.g. fhevmOperations1.ts:137-150: add(71, 66) == 137).  Every overload is kept: ebool and
(e)uint8 / 16 / 32 / 64 / 128 / 256 (2,394 KATs).  Clear values are written as decimal strings (the
256-bit ones do not survive a JSON number in JS); consumers read them with int() / BigInt().

    python tests/golden/extract_fhevm_kats.py  ->  tests/golden/fhevm_kats.json
"""
import glob
import json
import os
import re

SRC = "/root/reference/tests/fhevm-suite/e2e/test/fhevmOperations"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fhevm_kats.json")
KEEP = {"ebool"} | {f"{e}uint{w}" for e in ("", "e") for w in (8, 16, 32, 64, 128, 256)}
TITLE = re.compile(r"it\('test operator \"(\w+)\" overload \(([^)]*)\) => (\w+) test (\d+) \(([^)]*)\)'")
EXPECT = re.compile(r"expect\(res\)\.to\.equal\(([^)]*)\)")


def main():
    kats = []
    for path in sorted(glob.glob(os.path.join(SRC, "fhevmOperations*.ts"))):
        text = open(path).read()
        lines = text.splitlines()
        for i, line in enumerate(lines):
            m = TITLE.search(line)
            if not m:
                continue
            op, types, tres, num, args = m.groups()
            tys = [t.strip() for t in types.split(",")]
            if not all(t in KEEP for t in tys + [tres]):
                continue
            vals = [a.strip() for a in args.split(",")]
            exp = None
            for j in range(i + 1, min(i + 25, len(lines))):
                e = EXPECT.search(lines[j])
                if e:
                    exp = e.group(1).strip()
                    break
            if exp is None:
                continue
            exp = exp.rstrip("n")
            exp = {"true": 1, "false": 0}.get(exp, exp)
            kats.append({"op": op, "types": tys, "result_type": tres, "test": int(num),
                         "args": [str(int(v.rstrip("n"))) if v not in ("true", "false") else str(int(v == "true"))
                                  for v in vals],
                         "expect": str(int(exp)), "source": f"{os.path.basename(path)}:{i + 1}"})
    json.dump(kats, open(OUT, "w"), indent=0)
    ops = sorted(set(k["op"] for k in kats))
    print(f"{len(kats)} KATs, operators: {ops}")


if __name__ == "__main__":
    main()
