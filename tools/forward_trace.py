"""One graph replay of a model forward from a rocprofv3 kernel trace: the last `n` dispatches in
start order, each with its duration and the idle gap before it (offline analysis of
gpurun_out/*/run_kernel_trace.csv; tuning aid).

    python tools/forward_trace.py TRACE N
"""
import csv
import sys


def main(trace, n):
    rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))[-n:]
    t0, prev_end, busy = int(rows[0]["Start_Timestamp"]), None, 0
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = 0 if prev_end is None else s - prev_end
        busy += e - s
        print("%8.1f us  dur %7.2f  gap %6.2f  %s" % ((s - t0) / 1e3, (e - s) / 1e3, gap / 1e3,
                                                    r["Kernel_Name"][:110]))
        prev_end = e
    wall = (prev_end - t0) / 1e3
    print("wall %.1f us, kernel busy %.1f us (%.0f %%), %d dispatches" % (wall, busy / 1e3, 100.0 * busy / 1e3 / wall, n))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]))
