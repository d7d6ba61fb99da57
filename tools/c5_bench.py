"""C5 wall time on one MI355X (BASELINE.json configs[4]: the blind-auction FheUint32 max tree over 256 bidders,
chained PBS levels): 255 comparisons + selects in lockstep levels, one Engine.pbs launch per circuit level.

Timed: the whole tree after one untimed warm-up tree (host-side bit encryption of the bids is outside), from
the first launch to the device synchronisation after the last; `value` is the MEDIAN over --reps warm trees
(default 5), min / max beside it.  Every launch's batch size and time are recorded: for the device-resident
circuit a pair of HIP events around each pbs_device launch on torch's current stream (the stream the library
enqueues on), read after the tree's final synchronisation; for the host-array circuit the call's wall time incl.
transfers.  Default: the device-resident circuit (round 4); --host: the round-3 host-array circuit.
Prints ONE JSON line.
  python tools/c5_bench.py [--bidders 256] [--preset gate_fft|gate] [--reps 5] [--host]"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tfhe_amd  # noqa: E402
from tfhe_amd import integer as I  # noqa: E402
from tfhe_amd.auction import max_tree  # noqa: E402


class _Timed:
    """Engine proxy that records (batch, ms) of every pbs call."""

    def __init__(self, eng):
        self._e, self.calls, self._ev = eng, [], []

    def pbs_device(self, d_in, d_lut):
        # device-resident circuit: launches are queued, not waited for; events on the launch stream time them
        import torch
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        out = self._e.pbs_device(d_in, d_lut)
        e1.record()
        self._ev.append((int(d_in.shape[0]), e0, e1))
        return out

    def resolve(self):
        """after the final synchronisation: the device launches' (batch, ms) from their events"""
        self.calls += [(b, round(e0.elapsed_time(e1), 3)) for b, e0, e1 in self._ev]
        self._ev = []

    def pbs(self, cts, lut, idx=None):
        t = time.perf_counter()
        out = self._e.pbs(cts, lut) if idx is None else self._e.pbs(cts, lut, idx)
        self.calls.append((int(cts.shape[0]), round((time.perf_counter() - t) * 1e3, 3)))
        return out

    def __getattr__(self, k):
        return getattr(self._e, k)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bidders", type=int, default=256)
    ap.add_argument("--preset", choices=["gate_fft", "gate"], default="gate_fft")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--host", action="store_true",
                    help="host-array circuit (numpy, one H2D + D2H per level) instead of the device-resident one")
    a = ap.parse_args()
    p = tfhe_amd.Params.preset(tfhe_amd.PRESET_GATE_FFT if a.preset == "gate_fft" else tfhe_amd.PRESET_GATE)
    ck, sk = tfhe_amd.gen_keys(p, 0x7F4E0001)
    eng = tfhe_amd.Engine(p, 0).load_keys(sk)
    v = np.random.default_rng(5).integers(0, 2**32, a.bidders, dtype=np.uint64)
    v[min(77, a.bidders - 1)] = np.uint64(2**32 - 3)
    runs = []
    dev = None if a.host else "cuda:0"
    if dev:
        import torch
    for rep in range(a.reps + 1):
        te = _Timed(eng)
        c = I.Circuit(te, device=dev)
        bids = I.FheUint.encrypt(c, ck, v, 32, seed=0xB1D + rep, stream0=0)
        if dev:
            torch.cuda.synchronize()
        t = time.perf_counter()
        mx, idx = max_tree(c, bids)
        if dev:
            torch.cuda.synchronize()
        wall = time.perf_counter() - t
        te.resolve()
        ok = int(mx.decrypt(ck)[0]) == int(v.max()) and int(idx.decrypt(ck)[0]) == int(np.argmax(v))
        runs.append({"wall_s": round(wall, 4), "pbs": c.pbs_count, "launches": c.launches, "ok": ok,
                     "calls": te.calls})
    timed = runs[1:]
    walls = sorted(r["wall_s"] for r in timed)
    med = timed[[r["wall_s"] for r in timed].index(walls[len(walls) // 2])]  # the median run (odd reps: exact)
    print(json.dumps({
        "metric": f"C5 max-tree wall time, {a.bidders} FheUint32 bidders (255 comparisons + selects), 1 GPU",
        "circuit": "host arrays" if a.host else "device-resident (int64 tensors on the GPU, pbs_async per level)",
        "value": med["wall_s"], "stat": f"median of {len(timed)} warm trees", "min_s": walls[0], "max_s": walls[-1],
        "unit": "s", "higher_is_better": False, "preset": a.preset,
        "engine_kernels": {"lat_max": "per-shard batches <= the latency threshold run the latency kernel",
                           "pbs_ms_sum": round(sum(ms for _, ms in med["calls"]), 1),
                           "timing": "host wall incl. transfers" if a.host else "HIP events around each launch"},
        "walls_s": [r["wall_s"] for r in timed], "warmup_wall_s": runs[0]["wall_s"],
        "pbs": med["pbs"], "launches": med["launches"], "decrypt_ok": all(r["ok"] for r in runs),
        "launch_batches_ms": med["calls"]}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
