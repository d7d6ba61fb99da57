"""Summarize rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into profiles/<name>.json.

FETCH_SIZE / WRITE_SIZE are in KB.  gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE reads
exactly 1/2 of the bytes of a wide coalesced streaming read -> doubled here (our BSK stream is 8 B per
lane, an access width the guide lists as uncalibrated; the factor is applied as prescribed and noted).
WRITE_SIZE is exact for streaming stores (checked: blind-rotate writes 4096 x 8,200 B).

  python tools/pmc_summary.py gpurun_out/pmc_fetch gpurun_out/pmc_write profiles/r01_pmc_blind_rotate.json
"""
import csv
import json
import sys


def per_kernel(path):
    rows = list(csv.DictReader(open(path + "/run_counter_collection.csv")))
    agg = {}
    for r in rows:
        k = (r["Kernel_Name"].replace("(anonymous namespace)", "anon").split("(")[0], r["Counter_Name"])
        agg.setdefault(k, []).append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


def main(fetch_dir, write_dir, out):
    f, w = per_kernel(fetch_dir), per_kernel(write_dir)
    res = {}
    for (kern, cnt), v in list(f.items()) + list(w.items()):
        res.setdefault(kern, {})[cnt + "_KB"] = v
    for kern, d in res.items():
        fb = d.get("FETCH_SIZE_KB", 0.0) * 1024 * 2
        wb = d.get("WRITE_SIZE_KB", 0.0) * 1024
        d["hbm_bytes_per_launch"] = fb + wb
        d["note"] = "FETCH_SIZE x2 (gfx950 correction) + WRITE_SIZE, bytes per launch"
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:4])
