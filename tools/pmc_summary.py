"""Summarize rocprofv3 PMC passes (tools/pmc_profile.sh) into profiles/pmc_<workload>.json.

    python tools/pmc_summary.py <pmc run dir> <workload> <kernel substring[;substring...]> [out.json]

Several ";"-separated substrings (kernel names contain commas): the per-launch figures are the SUM over those kernels
(e.g. one LightGCN propagation layer = spmm_light + spmm_segment + spmm_finish).  A
substring ending in "@max" keeps only that kernel's dispatches with its largest grid (the
whole-graph SpMM layers, not the restricted last layer's row-range launches).

HBM traffic per launch of the dominant kernel, corrected as MI355X_MICROARCH.md's
HBM/rocprofv3 section prescribes: FETCH_SIZE (kB) counts L2 -> fabric read requests and on
gfx950 reports exactly half the bytes of 16-B-per-lane streaming reads, so it is doubled;
WRITE_SIZE (kB) reads 16-B stores exactly.  Infinity-Cache hits are included (memory-side
counters), so this is "bytes that left the L2", an upper bound of HBM bytes.
"""
import collections
import csv
import glob
import json
import os
import sys


def main():
    run, workload, ksub = sys.argv[1], sys.argv[2], sys.argv[3]
    out = sys.argv[4] if len(sys.argv) > 4 else os.path.join("profiles", f"pmc_{workload}.json")
    subs = ksub.split(";")
    per = {sub: collections.defaultdict(list) for sub in subs}
    names = set()
    rows = []
    for f in sorted(glob.glob(os.path.join(run, "p*", "*counter_collection.csv"))):
        rows += list(csv.DictReader(open(f)))
    maxgrid = {}
    for r in rows:
        for sub in subs:
            if sub.endswith("@max") and sub[:-4] in r["Kernel_Name"]:
                maxgrid[sub] = max(maxgrid.get(sub, 0), int(r["Grid_Size"]))
    for r in rows:
        for sub in subs:
            key = sub[:-4] if sub.endswith("@max") else sub
            if key in r["Kernel_Name"]:
                if sub in maxgrid and int(r["Grid_Size"]) != maxgrid[sub]:
                    break
                names.add(r["Kernel_Name"])
                per[sub][r["Counter_Name"]].append(float(r["Counter_Value"]))
                break
    if not any(per.values()):
        raise SystemExit(f"no dispatches of a kernel matching {ksub!r} under {run}")
    avg = collections.defaultdict(float)  # per-launch sum over the listed kernels
    vals = collections.defaultdict(list)
    for sub, d in per.items():
        for k, v in d.items():
            avg[k] += sum(v) / len(v)
            vals[k] += v
    avg = dict(avg)
    fetch = 2.0 * avg.get("FETCH_SIZE", 0.0) * 1024.0   # kB -> B, x2 gfx950 correction
    write = avg.get("WRITE_SIZE", 0.0) * 1024.0
    clk = avg.get("GRBM_GUI_ACTIVE", 0.0) / 8.0        # summed over the 8 XCDs
    simd = 1024.0
    summary = {
        "workload": workload,
        "kernel": sorted(names),
        "dispatches_per_counter": {k: len(v) for k, v in vals.items()},
        "hbm_bytes_per_launch": fetch + write,
        "fetch_bytes_per_launch": fetch,
        "write_bytes_per_launch": write,
        "correction": "FETCH_SIZE x2 (gfx950 16-B/lane reads), kB -> bytes; includes MALL hits",
        "gpu_cycles_per_launch": clk,
        "mfma_busy_frac": avg.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / simd / clk if clk else None,
        "valu_insts_per_simd": avg.get("SQ_INSTS_VALU", 0.0) / simd,
        "mfma_insts_per_simd": avg.get("SQ_INSTS_MFMA", 0.0) / simd,
        "lds_bank_conflicts": avg.get("SQ_LDS_BANK_CONFLICT"),
        "raw_counter_means": avg,
    }
    os.makedirs(os.path.dirname(out) or ".", exist_ok=True)
    json.dump(summary, open(out, "w"), indent=1)
    print(json.dumps({k: summary[k] for k in ("workload", "hbm_bytes_per_launch",
                                               "mfma_busy_frac", "gpu_cycles_per_launch")}))


if __name__ == "__main__":
    main()
