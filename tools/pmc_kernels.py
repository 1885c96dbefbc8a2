"""Per-kernel means of every counter in rocprofv3 --pmc runs (counter_collection.csv under the
given directories), for kernels whose name contains any of the given substrings.

    python tools/pmc_kernels.py "<substr>[;<substr>...]" <run dir> [<run dir> ...]
"""
import collections
import csv
import glob
import os
import sys


def main():
    subs = sys.argv[1].split(";")
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in sys.argv[2:]:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                name = r["Kernel_Name"]
                if any(s in name for s in subs):
                    key = (name.split("(")[0][-60:], int(r["Grid_Size"]))
                    acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for (name, grid), cs in sorted(acc.items()):
        parts = [f"{c}={sum(v) / len(v):.4g}(n={len(v)})" for c, v in sorted(cs.items())]
        extra = ""
        if "TCC_HIT_sum" in cs and "TCC_MISS_sum" in cs:
            h = sum(cs["TCC_HIT_sum"]) / len(cs["TCC_HIT_sum"])
            m = sum(cs["TCC_MISS_sum"]) / len(cs["TCC_MISS_sum"])
            extra = f" L2hit={h / max(h + m, 1):.3f}"
        if "FETCH_SIZE" in cs:
            extra += f" fetchGB={2 * 1024 * sum(cs['FETCH_SIZE']) / len(cs['FETCH_SIZE']) / 1e9:.3f}"
        print(f"{name} grid={grid}: " + " ".join(parts) + extra)


if __name__ == "__main__":
    main()
