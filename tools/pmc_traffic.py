"""HBM traffic per launch of one kernel from tools/pmc.sh's FETCH_SIZE (pass 1) and WRITE_SIZE (pass 2)
rocprofv3 runs, corrected as MI355X_MICROARCH.md's HBM/rocprofv3 section prescribes:
  - the counters are in KiB;
  - on gfx950 FETCH_SIZE reports half the bytes of a coalesced streaming read, so it is doubled;
  - WRITE_SIZE is exact for coalesced stores.
The result is merged into profiles/traffic.json under the bench workload key; bench.py reports it as
`roofline.traffic` when its dominant kernel is the same one.

usage: python tools/pmc_traffic.py <pmc-dir> <kernel-regex> <timer-name> <query> [--out profiles/traffic.json]
"""
import argparse
import csv
import json
import os
import re


def dispatches(path, counter, kre):
    """The counter's value per dispatch of the kernel, in dispatch order (summed over rows of one
    dispatch: a counter may be reported per XCD or per instance)."""
    by = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter and re.search(kre, r["Kernel_Name"]):
            k = int(r.get("Dispatch_Id") or r.get("Correlation_Id") or len(by))
            by[k] = by.get(k, 0.0) + float(r["Counter_Value"])
    if not by:
        raise SystemExit("no %s rows for %s in %s" % (counter, kre, path))
    return [by[k] for k in sorted(by)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("pmc_dir")
    ap.add_argument("kernel_regex")
    ap.add_argument("timer_name")
    ap.add_argument("query")
    ap.add_argument("--out", default=os.path.join(os.path.dirname(__file__), "..", "profiles", "traffic.json"))
    a = ap.parse_args()
    f = dispatches(os.path.join(a.pmc_dir, "p1", "pmc_counter_collection.csv"), "FETCH_SIZE", a.kernel_regex)
    w = dispatches(os.path.join(a.pmc_dir, "p2", "pmc_counter_collection.csv"), "WRITE_SIZE", a.kernel_regex)
    if len(f) != len(w):
        raise SystemExit("dispatch counts differ between the passes: %d vs %d" % (len(f), len(w)))
    # a kernel launched several times per step with very different sizes (M1: the first hop, then the
    # row emission) is reported on its main launches: those moving at least half the largest one's bytes
    tot = [2 * x + y for x, y in zip(f, w)]
    main = [i for i, t in enumerate(tot) if t >= 0.5 * max(tot)]
    fetch = sum(f[i] for i in main) / len(main)
    write = sum(w[i] for i in main) / len(main)
    rec = {"kernel": a.timer_name, "fetch_size_kib": fetch, "write_size_kib": write,
           "read_bytes": 2 * fetch * 1024, "write_bytes": write * 1024,
           "bytes_per_launch": 2 * fetch * 1024 + write * 1024, "dispatches": [len(f), len(main)],
           "dispatches_note": "[all dispatches of the kernel, main dispatches averaged]",
           "source": os.path.relpath(a.pmc_dir, os.path.join(os.path.dirname(__file__), ".."))}
    db = json.load(open(a.out)) if os.path.exists(a.out) else {}
    db[a.query] = rec
    with open(a.out, "w") as f:
        json.dump(db, f, indent=1, sort_keys=True)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
