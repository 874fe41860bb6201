"""Interleaved A/B of env-switch variants on one box: `python3 tools/ab.py OUT REPS QUERY VAR=VAL[,VAR=VAL] ...`
(a variant "-" is the default build). Each repetition runs bench.py once per variant (no CPU baseline, no
deliver), 20 timed steps; prints ms_per_step and the main kernels per run, then the median per variant,
and writes OUT/ab.json. Every run is bounded by its own timeout; a failing run ends the script."""
import json
import os
import statistics
import subprocess
import sys


def main():
    out, reps, query, variants = sys.argv[1], int(sys.argv[2]), sys.argv[3], sys.argv[4:]
    os.makedirs(out, exist_ok=True)
    res = {v: [] for v in variants}
    for r in range(reps):
        for v in variants:
            env = dict(os.environ)
            if v != "-":
                for kv in v.split(","):
                    k, x = kv.split("=", 1)
                    env[k] = x
            cmd = ["timeout", "-k", "10", "240", sys.executable, "bench.py", "--query", query, "--steps", "20",
                   "--warmup", "5", "--no-cpu-baseline", "--no-deliver"]
            p = subprocess.run(cmd, env=env, capture_output=True, text=True)
            if p.returncode != 0:
                print("FAILED", v, p.returncode, p.stderr[-2000:])
                sys.exit(1)
            d = json.loads(p.stdout.strip().splitlines()[-1])
            ks = {k: round(x["ms_per_step"], 3) for k, x in list(d["kernels"].items())[:4]}
            res[v].append({"ms": d["ms_per_step"], "kernels": ks, "step_kernel_ms": d["roofline"]["step_kernel_ms"]})
            print("rep %d %-40s %.3f ms  kernels %s" % (r, v, d["ms_per_step"], ks), flush=True)
    for v in variants:
        print("median %-40s %.3f ms" % (v, statistics.median(x["ms"] for x in res[v])))
    json.dump(res, open(os.path.join(out, "ab.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
