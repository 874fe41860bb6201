"""One-screen summary of a bench.py JSON line (and, given a rocprofv3 output directory, its top kernels
by total time). usage: python tools/summarize.py <bench.json> [<rocprof dir>]"""
import csv
import glob
import json
import os
import sys


def main():
    d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
    r = d.get("roofline") or {}
    print("%s: %.1f %s  %.3f ms/step  read %.1f G/s  | %s launch %.3f ms %.2f GB -> %.0f GB/s frac %.3f | step_frac %.3f"
          % (d["config"].get("workload", "")[:40], d["value"], d["unit"], d["ms_per_step"],
             (d.get("read_rate") or {}).get("value", 0.0), r.get("kernel"), r.get("avg_launch_ms", 0),
             r.get("alg_bytes_per_launch", 0) / 1e9, r.get("achieved", 0), r.get("frac", 0), r.get("step_frac", 0)))
    ks = d.get("kernels", {})
    print("  kernels (ms/step): " + ", ".join("%s %.3f" % (k, v["ms_per_step"]) for k, v in list(ks.items())[:8]))
    if d.get("cpu_baseline"):
        c = d["cpu_baseline"]
        print("  cpu_baseline: %.3f %s on %s threads" % (c["value"], c["unit"], c["cores"]))
        if c.get("set_based"):
            print("  cpu_baseline set_based: %.3f %s on %s threads" % (c["set_based"]["value"], c["set_based"]["unit"],
                                                                      c["set_based"]["cores"]))
    if len(sys.argv) > 2:
        f = glob.glob(os.path.join(sys.argv[2], "**", "*kernel_stats.csv"), recursive=True)
        if f:
            rows = sorted(csv.DictReader(open(f[0])), key=lambda x: -float(x["TotalDurationNs"]))
            for x in rows[:10]:
                print("  rocprof %-60s calls %6s avg %9.1f us total %9.2f ms" % (
                    x["Name"][:60], x["Calls"], float(x["AverageNs"]) / 1e3, float(x["TotalDurationNs"]) / 1e6))


if __name__ == "__main__":
    main()
