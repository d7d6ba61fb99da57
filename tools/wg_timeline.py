"""Per-workgroup timeline of one batch blind rotation, P-GATE or P-FHEVM (diagnostic build only:
make -C tfhe_amd B=../build_diag/wgt/obj LIB=../build_diag/wgt/libtfhe_hip.so EXTRA=-DFFT_WGTIME=1, run with
TFHE_HIP_LIB=build_diag/wgt/libtfhe_hip.so on the GPU box).

Reads each workgroup's start / end (s_memrealtime, 100 MHz), HW_ID and XCC_ID of the last launch and prints where the
launch's time goes: workgroup durations, the dispatch rounds, and the drain (CU-slot time left idle after a slot's
last workgroup while the launch is still running).
  python tools/wg_timeline.py [--preset gate_fft|fhevm_fft] [--batch 4096] [--out gpurun_out/wg_timeline.json]"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tfhe_amd  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--out", default="gpurun_out/wg_timeline.json")
    ap.add_argument("--preset", choices=["gate_fft", "fhevm_fft"], default="gate_fft")
    a = ap.parse_args()
    import torch
    fhevm = a.preset == "fhevm_fft"
    params = tfhe_amd.Params.preset(tfhe_amd.PRESET_FHEVM_FFT if fhevm else tfhe_amd.PRESET_GATE_FFT)
    ck, sk = tfhe_amd.gen_keys(params, 0x7F4E0001)
    eng = tfhe_amd.Engine(params, 0).load_keys(sk)
    B = a.batch
    if fhevm:
        eng.load_ms_key(tfhe_amd.ms_zeros_keygen(params, 0x7F4E0001, ck.lwe_key))
        cts = ck.encrypt((np.arange(B) % 16).astype(np.uint64), 16, seed=0xC0FFEE01)
        lut = eng.generate_accumulator(lambda m: m, 16)
    else:
        bits = np.random.default_rng(1).integers(0, 2, B).astype(bool)
        cts = ck.encrypt_bool(bits, seed=0xC0FFEE01)
        lut = eng.gate_lut()
    dev = torch.device("cuda:0")
    d_in = torch.from_numpy(cts.view(np.int64)).to(dev)
    d_lut = torch.from_numpy(lut.view(np.int64)).to(dev)
    d_out = torch.empty_like(d_in)
    for _ in range(4):
        eng.pbs_async(d_in, d_lut, d_out)
    torch.cuda.synchronize()
    L = tfhe_amd.lib()
    nwg = (B + 1) // 2
    buf = np.zeros(4 * 16384, dtype=np.uint64)
    fn = L.tfhe_hip_debug_wgtimes2k if fhevm else L.tfhe_hip_debug_wgtimes
    fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    assert fn(buf.ctypes.data, buf.size) == 0
    t = buf[: 4 * nwg].reshape(nwg, 4)
    t0, t1 = t[:, 0].astype(np.int64), t[:, 1].astype(np.int64)
    base = t0.min()
    s_us, e_us = (t0 - base) / 100.0, (t1 - base) / 100.0   # 100 MHz -> us
    dur = e_us - s_us
    hw, xcc = t[:, 2].astype(np.int64), t[:, 3].astype(np.int64) & 0xF
    cu = (hw >> 8) & 0xF
    sh_ = (hw >> 12) & 1
    se = (hw >> 13) & 0x7
    slot_key = xcc * 1000 + se * 100 + sh_ * 20 + cu          # one key per CU
    span = e_us.max()
    res = {"batch": B, "workgroups": nwg, "span_us": round(float(span), 1),
           "dur_us": {"mean": round(float(dur.mean()), 1), "min": round(float(dur.min()), 1),
                      "max": round(float(dur.max()), 1), "p10": round(float(np.percentile(dur, 10)), 1),
                      "p90": round(float(np.percentile(dur, 90)), 1)},
           "cus_seen": int(len(np.unique(slot_key)))}
    # per CU: busy time = sum of its workgroups' durations / 2 slots; the CU's last end
    per = {}
    for k, s0, e0, d in zip(slot_key, s_us, e_us, dur):
        p = per.setdefault(int(k), [0.0, 0.0, 0])
        p[0] += d
        p[1] = max(p[1], e0)
        p[2] += 1
    last = np.array([v[1] for v in per.values()])
    busy = np.array([v[0] for v in per.values()])
    cnt = np.array([v[2] for v in per.values()])
    res["per_cu"] = {"wgs_min": int(cnt.min()), "wgs_max": int(cnt.max()),
                     "last_end_us": {"min": round(float(last.min()), 1), "median": round(float(np.median(last)), 1),
                                     "max": round(float(last.max()), 1)},
                     "busy_over_2span": round(float(busy.sum() / (2 * span * len(per))), 4)}
    # dispatch rounds: start-time histogram of the workgroups (first 512 start at ~0)
    order = np.argsort(s_us)
    res["first_round_start_spread_us"] = round(float(s_us[order[:512]].max()), 1)
    res["start_quantiles_us"] = [round(float(np.percentile(s_us, q)), 1) for q in (0, 25, 50, 75, 100)]
    res["per_xcc_span_us"] = {int(x): round(float(e_us[xcc == x].max()), 1) for x in np.unique(xcc)}
    res["per_xcc_mean_dur_us"] = {int(x): round(float(dur[xcc == x].mean()), 1) for x in np.unique(xcc)}
    # the two workgroup slots of each CU (a workgroup takes the slot whose previous workgroup ended closest to its
    # start): how far apart the slots' last workgroups end
    by_cu = {}
    for i, k in enumerate(slot_key):
        by_cu.setdefault(int(k), []).append((s_us[i], e_us[i]))
    diffs = []
    for v in by_cu.values():
        v.sort()
        if len(v) < 2:
            continue
        ends = [v[0][1], v[1][1]]
        for st, en in v[2:]:
            j = 0 if abs(ends[0] - st) < abs(ends[1] - st) else 1
            ends[j] = en
        diffs.append(abs(ends[0] - ends[1]))
    res["slot_end_diff_us"] = {"mean": round(float(np.mean(diffs)), 1), "max": round(float(np.max(diffs)), 1)}
    res["wg0_16"] = [[int(slot_key[i]), round(float(s_us[i]), 1), round(float(e_us[i]), 1)] for i in range(16)]
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    json.dump(res, open(a.out, "w"), indent=1)
    np.save(a.out.replace(".json", ".npy"), t)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
