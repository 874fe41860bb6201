"""Print the last N kernel dispatches of a rocprofv3 kernel trace with their durations and the idle gaps
between them (development aid: where a bench step's time goes besides the big kernels).

usage: python tools/timeline.py gpurun_out/prof/c2_kernel_trace.csv [N]
"""
import csv
import sys


def main():
    path = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 60
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    rows = rows[-n:]
    prev_end = None
    busy = 0
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s - prev_end) / 1e3 if prev_end is not None else 0.0
        busy += e - s
        name = r["Kernel_Name"].split("(")[0][:60]
        print("%8.1f gap  %8.1f us  grid %9s  %s" % (gap, (e - s) / 1e3, r["Grid_Size_X"], name))
        prev_end = e
    span = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1e3
    print("span %.1f us, busy %.1f us" % (span, busy / 1e3))


if __name__ == "__main__":
    main()
