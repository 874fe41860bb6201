"""Per-kernel averages of every counter in a tools/pmc.sh output directory (development aid).

usage: python tools/pmc_summary.py <pmc-dir> [kernel-regex]
"""
import csv
import glob
import os
import re
import sys


def main():
    d = sys.argv[1]
    kre = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
    acc = {}
    for f in sorted(glob.glob(os.path.join(d, "p*", "pmc_counter_collection.csv"))):
        per = {}
        for r in csv.DictReader(open(f)):
            name = re.sub(r"\(anonymous namespace\)::", "", r["Kernel_Name"]).split("(")[0][-48:]
            if kre and not kre.search(r["Kernel_Name"]):
                continue
            key = (name, r["Counter_Name"], r.get("Dispatch_Id") or r.get("Correlation_Id"))
            per[key] = per.get(key, 0.0) + float(r["Counter_Value"])
        for (name, c, _), v in per.items():
            a = acc.setdefault((name, c), [0.0, 0])
            a[0] += v
            a[1] += 1
    for (name, c), (v, n) in sorted(acc.items()):
        print("%-48s %-24s %16.4g  (%d dispatches)" % (name, c, v / n, n))


if __name__ == "__main__":
    main()
