"""Cut a host-clock window out of a rocprofv3 kernel trace and summarise it per kernel.

    python tools/trace_window.py <kernel_trace.csv> <window.json> <out.txt>

window.json is the line tools/bench_d4.py --lstm-trace printed ({"chunks": K, "window_ns":
{clock: [t0, t1]}}): the kernels whose start lies in [t0, t1] on the clock that brackets
them (rocprofv3 stamps kernels on one of the host clocks) are grouped by name, with their
launches and GPU time per chunk, in descending time order."""
import collections
import csv
import json
import sys


def main(trace, window, out):
    w = json.loads(open(window).read().strip().splitlines()[-1])
    rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
            for r in csv.DictReader(open(trace))]
    best = None
    for clock, (t0, t1) in w["window_ns"].items():
        sel = [r for r in rows if t0 <= r[0] <= t1]
        if sel and (best is None or len(sel) > len(best[1])):
            best = (clock, sel, t0, t1)
    if best is None:
        raise SystemExit("no kernel of the trace lies in the window on any clock")
    clock, sel, t0, t1 = best
    k = w["chunks"]
    per = collections.defaultdict(lambda: [0, 0])
    for s, e, n in sel:
        per[n][0] += 1
        per[n][1] += e - s
    busy = sum(v[1] for v in per.values())
    lines = ["# %d chunks of %d tokens, clock %s, window %.3f ms/chunk (host), kernels %.3f "
             "ms/chunk (GPU busy), %d launches/chunk" % (
                 k, w["tokens_per_chunk"], clock, (t1 - t0) / k / 1e6, busy / k / 1e6,
                 len(sel) // k),
             "%-10s %-10s %-10s %-7s %s" % ("us/chunk", "launches", "us/launch", "share",
                                            "kernel")]
    for n, (c, d) in sorted(per.items(), key=lambda kv: -kv[1][1]):
        lines.append("%-10.1f %-10.2f %-10.2f %-7.3f %s" % (
            d / k / 1e3, c / k, d / c / 1e3, d / busy, n[:160]))
    open(out, "w").write("\n".join(lines) + "\n")
    print("\n".join(lines[:14]))


if __name__ == "__main__":
    main(*sys.argv[1:4])
