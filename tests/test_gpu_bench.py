"""bench.py keeps the driver's contract: one JSON line with the metric, the whole-job value, the
roofline and cpu_baseline objects, and a bit-exact oracle comparison of the sampled outputs
(run here at a reduced batch so it takes seconds; the round-end bench runs the full 4096)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("preset", ["gate_fft", "fhevm_fft"])
def test_bench_json_contract(preset):
    r = subprocess.run([sys.executable, "bench.py", "--preset", preset, "--steps", "2", "--warmup", "1",
                        "--batch", "512", "--cpu-sample", "32"], cwd=ROOT, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.strip().startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 2 and d["warmup"] == 1 and d["value"] > 0
    assert d["dtype"] == "f64" and d["config"]["batch_per_gpu"] == 512
    rf = d["roofline"]
    # VALU-issue bound; at B = 512 no same-build counter profile exists, so the f64 FLOP figure is reported
    assert rf["bound"] == "valu" and rf["kernel_ms"] > 0
    assert rf["unit"] == "TFLOP/s" and rf["peak"] == 78.6 and rf["traffic"] is None
    assert abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-3 and 0 < rf["frac"] <= 1
    assert rf["hbm_model_r1"]["bytes_per_launch"] > 0
    cb = d["cpu_baseline"]
    assert cb["kind"] == "port" and cb["cores"] >= 1 and cb["value"] > 0
    assert d["decrypt_ok"] is True and d["sample_bitexact"] is True
    bx = d["bitexact_check"]
    assert bx["bitexact_pbs"] == 32 and bx["gpu_sha256"] == bx["oracle_sha256"]


def test_bench_strong_scaling_mode():
    """--global-batch: one global batch, this rank's contiguous slice, scaling "strong"."""
    r = subprocess.run([sys.executable, "bench.py", "--steps", "1", "--warmup", "1", "--global-batch", "1024",
                        "--no-cpu"], cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.strip().startswith("{")][0])
    assert d["scaling"] == "strong" and d["config"]["global_batch"] == 1024 and d["config"]["batch_per_gpu"] == 1024
    assert d["decrypt_ok"] is True


def test_bench_c3_config():
    """--config c3 (BASELINE.json configs[2]): FheUint8 values x 8 per-bit LUTs in one multi-LUT launch; every byte
    decrypted, the CPU sample (whole FheUint8 values, lut_index included) bit-exact against the oracle."""
    r = subprocess.run([sys.executable, "bench.py", "--config", "c3", "--steps", "2", "--warmup", "1", "--batch", "128",
                        "--cpu-sample", "64"], cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.strip().startswith("{")][0])
    assert d["unit"] == "FheUint8/s" and d["config"]["batch_per_gpu"] == 128 and d["config"]["pbs_per_gpu"] == 1024
    assert abs(d["pbs_per_s"] - 8 * d["value"]) < 1e-6 * d["pbs_per_s"] + 1
    assert d["decrypt_ok"] is True and d["sample_bitexact"] is True
    assert d["roofline"]["launches"] == 2 and d["roofline"]["kernel_ms"] > 0
    bx = d["bitexact_check"]
    assert bx["bitexact_pbs"] == 64 and bx["gpu_sha256"] == bx["oracle_sha256"]
