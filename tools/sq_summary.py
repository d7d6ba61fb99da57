"""Per-kernel averages of a rocprofv3 SQ counter pass (counter_collection.csv) with derived ratios.

  python tools/sq_summary.py gpurun_out/r01_fft1_pmc_sq.csv [kernel-substring]
"""
import csv
import sys


def main(path, sub="blind_rotate"):
    agg = {}
    for r in csv.DictReader(open(path)):
        if sub not in r["Kernel_Name"]:
            continue
        k = r["Kernel_Name"].split("(")[0]
        agg.setdefault(k, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    for k, d in agg.items():
        v = {c: sum(x) / len(x) for c, x in d.items()}
        print(k)
        for c in sorted(v):
            print(f"  {c:24s} {v[c]:.4g}")
        wc = v.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS"):
                if c in v:
                    print(f"  {c + ' / WAVE_CYCLES':40s} {v[c] / wc:.3f}")


if __name__ == "__main__":
    main(*sys.argv[1:])
