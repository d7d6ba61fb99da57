"""Per-kernel roofline summary of one profiling session -> profiles/<tag>_roofline.json.

Inputs (all from the SAME tree, produced by tools/profile_round.sh on the GPU box):
  * rocprofv3 --kernel-trace --stats summary (kernel_stats.csv): average launch duration;
  * one SQ counter pass (counter_collection.csv): SQ_INSTS_VALU, SQ_WAVE_CYCLES, SQ_WAIT_*, GRBM_GUI_ACTIVE;
  * optionally an SQ instruction-mix pass (SQ_INSTS_VALU_{FMA,ADD,MUL}_F64, _INT32, _INT64, _CVT, ...);
  * FETCH_SIZE and WRITE_SIZE passes (separate runs: TCC budget).

Derived figures per kernel and launch:
  * valu_issue_frac = SQ_INSTS_VALU x 4 cycles / (1024 SIMDs x 2.4 GHz x avg launch time): the f64-rate
    issue model (a wave64 f64 VALU instruction occupies a 16-lane-f64 SIMD for 4 cycles; 78.6 TFLOP/s
    spec FP64 vector = 256 CUs x 4 SIMDs x 16 lanes x 2 x 2.4 GHz);
  * hbm_bytes = FETCH_SIZE x 2 (gfx950: FETCH_SIZE reports half the bytes of wide streaming reads,
    MI355X_MICROARCH.md section HBM) + WRITE_SIZE; FETCH_SIZE / WRITE_SIZE are in KB.
The tree's tfhe_amd.source_id() is stored with the numbers; bench.py uses them only when its own
source_id matches.

  python tools/roofline_summary.py TAG STATS_CSV SQ_CSV FETCH_CSV WRITE_CSV [MIX_CSV] OUT_JSON
"""
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def kname(s: str) -> str:
    s = s.replace("(anonymous namespace)", "anon")
    base = s.split("(")[0]
    return base.replace("void ", "").strip()


def counters(path):
    agg = {}
    if not path or not os.path.exists(path):
        return agg
    for r in csv.DictReader(open(path)):
        agg.setdefault(kname(r["Kernel_Name"]), {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in agg.items()}


def main(tag, stats_csv, sq_csv, fetch_csv, write_csv, *rest):
    out = rest[-1]
    mix_csv = rest[0] if len(rest) > 1 else None
    from tfhe_amd import source_id
    stats = {}
    for r in csv.DictReader(open(stats_csv)):
        stats[kname(r["Name"])] = {"launches": int(r["Calls"]), "avg_ms": float(r["AverageNs"]) * 1e-6}
    sq, mix, fe, wr = counters(sq_csv), counters(mix_csv), counters(fetch_csv), counters(write_csv)
    res = {"tag": tag, "source_id": source_id(), "batch": int(os.environ.get("BATCH", "4096")),
           "model": {"valu_issue": "SQ_INSTS_VALU x 4 / (1024 SIMDs x 2.4e9 Hz x avg_ms)",
                     "hbm_bytes": "FETCH_SIZE x 2 (gfx950 correction) + WRITE_SIZE, KB -> bytes"},
           "kernels": {}}
    for k, s in stats.items():
        d = dict(s)
        c = sq.get(k, {})
        d.update({n: v for n, v in c.items()})
        d.update({n: v for n, v in mix.get(k, {}).items()})
        if "SQ_INSTS_VALU" in c and s["avg_ms"] > 0:
            d["valu_issue_frac"] = round(c["SQ_INSTS_VALU"] * 4 / (1024 * 2.4e9 * s["avg_ms"] * 1e-3), 4)
        m = mix.get(k, {})
        f64 = sum(m.get(n, 0.0) for n in ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64",
                                          "SQ_INSTS_VALU_TRANS_F64"))
        if f64 and c.get("SQ_INSTS_VALU"):
            d["f64_share"] = round(f64 / c["SQ_INSTS_VALU"], 4)   # f64 share of the VALU instruction stream
        if "SQ_WAVE_CYCLES" in c:
            for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_ANY"):
                if n in c:
                    d[n + "_per_wave_cycle"] = round(c[n] / c["SQ_WAVE_CYCLES"], 4)
        if k in fe or k in wr:
            d["FETCH_SIZE_KB"] = fe.get(k, {}).get("FETCH_SIZE", 0.0)
            d["WRITE_SIZE_KB"] = wr.get(k, {}).get("WRITE_SIZE", 0.0)
            d["hbm_bytes"] = round(d["FETCH_SIZE_KB"] * 1024 * 2 + d["WRITE_SIZE_KB"] * 1024)
            if s["avg_ms"] > 0:
                d["hbm_GBps"] = round(d["hbm_bytes"] / (s["avg_ms"] * 1e-3) / 1e9, 1)
        res["kernels"][k] = d
    json.dump(res, open(out, "w"), indent=1)
    for k, d in res["kernels"].items():
        if "blind_rotate" in k or "ks_gemm" in k or "sns" in k:
            print(k, {n: d.get(n) for n in ("avg_ms", "valu_issue_frac", "hbm_bytes", "hbm_GBps")})


if __name__ == "__main__":
    main(*sys.argv[1:])
