"""ASan + UBSan over the host code: the CPU oracle and the product's client-side key material
(tfhe_amd/csrc/client.cpp) built with -fsanitize=address,undefined (oracle/Makefile target `san`) and
driven by tools/sanitize/san_check.cpp: keygen of both parameter sets (identical to the oracle's),
OS-entropy and seeded ChaCha keys, encryption, full oracle PBS on the NTT and FFT64 transforms with the
P-FHEVM modulus-switch reduction, decryption, packing key and compression.  Any sanitizer report aborts
the binary (-fno-sanitize-recover=all).  GPU sanitizers are not available on the GPU pool."""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT

ORACLE = os.path.join(ROOT, "oracle")


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")
def test_host_code_clean_under_asan_ubsan():
    subprocess.run(["make", "-s", "-C", ORACLE, "san"], check=True, timeout=600)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([os.path.join(ORACLE, "_san", "san_check")], capture_output=True, text=True, timeout=900,
                       env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert "SANITIZE OK" in r.stdout
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr
