"""Per-kernel time of the timed bench steps from a rocprofv3 kernel trace: the trace's last `steps`
steps (a step = the kernels from one launch of the first kernel of the step's sequence to the
next), aggregated by kernel name, per step.  Offline analysis of gpurun_out/*/run_kernel_trace.csv.

    python tools/step_breakdown.py gpurun_out/prof/run_kernel_trace.csv [--steps 5] [--first conv_pair<16]
"""
import argparse
import collections
import csv
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--per-step", type=int, default=9, help="calls of --first per step")
    ap.add_argument("--first", default="conv_pair_rs16<", help="a kernel called --per-step times per step")
    args = ap.parse_args()
    rows = list(csv.DictReader(open(args.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if args.first in r["Kernel_Name"]]
    need = args.steps * args.per_step
    if len(idx) < need + 1:
        raise SystemExit("trace holds %d calls of %s, need %d" % (len(idx), args.first, need + 1))
    # the window: from the first kernel after the call that ends step -(steps+1) to the end, trimmed
    # to the first call of the last `steps` steps .. the kernel before the next step's first call
    lo = idx[-need]
    # walk back to the step's first kernel: the kernels between the previous step's last pair and this one
    prev = idx[-need - 1]
    gaps = [int(rows[i + 1]["Start_Timestamp"]) - int(rows[i]["End_Timestamp"]) for i in range(prev, lo)]
    start = prev + 1 + max(range(len(gaps)), key=lambda k: gaps[k]) if gaps else lo
    span = rows[start:]
    tot, cnt = collections.Counter(), collections.Counter()
    for r in span:
        name = re.sub(r"\(.*", "", r["Kernel_Name"])
        tot[name] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        cnt[name] += 1
    wall = int(span[-1]["End_Timestamp"]) - int(span[0]["Start_Timestamp"])
    busy = sum(tot.values())
    print("window: %d kernels, wall %.3f ms, busy %.3f ms; per step (%d): wall %.3f busy %.3f ms"
          % (len(span), wall / 1e6, busy / 1e6, args.steps, wall / 1e6 / args.steps, busy / 1e6 / args.steps))
    for k, v in tot.most_common(25):
        print("%9.3f ms/step %6.1f calls/step %6.1f us/call  %5.1f%%  %s"
              % (v / 1e6 / args.steps, cnt[k] / args.steps, v / 1e3 / cnt[k], 100.0 * v / busy, k[:110]))


if __name__ == "__main__":
    main()
