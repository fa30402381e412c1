"""Per-kernel table of tools/gpu_d4_pmc.sh: launches, average duration (kernel trace), and
average FETCH_SIZE (x2, the gfx950 correction of MI355X_MICROARCH.md for 16-byte streaming
reads) / WRITE_SIZE per dispatch in MB, with the bytes/duration rate.
    python tools/d4_pmc_report.py gpurun_out/<tag>"""
import collections
import csv
import glob
import os
import sys


def short(name):
    for k in ("dwconv", "act_encode_act", "se_gate", "conv2d_tp", "stem", "pool", "gemm",
              "elementwise", "reduce"):
        if k in name:
            return k + ("" if k != "conv2d_tp" else ":" + name.split("<")[0].split("(")[0][-28:])
    return name.split("(")[0][:40]


def main():
    root = sys.argv[1]
    for arch in sorted(os.listdir(root)):
        d = os.path.join(root, arch)
        if not os.path.isdir(d):
            continue
        dur = collections.defaultdict(list)
        for f in glob.glob(os.path.join(d, "trace", "**", "*kernel_trace.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                dur[short(r["Kernel_Name"])].append(
                    (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        ctr = collections.defaultdict(list)
        for c in ("FETCH_SIZE", "WRITE_SIZE"):
            for f in glob.glob(os.path.join(d, c, "**", "*counter_collection.csv"),
                               recursive=True):
                for r in csv.DictReader(open(f)):
                    ctr[(short(r["Kernel_Name"]), c)].append(float(r["Counter_Value"]))
        print("== %s" % arch)
        print("%-44s %7s %9s %10s %10s %8s" % ("kernel", "n", "avg_us", "fetch_MB", "write_MB",
                                               "GB/s"))
        for k in sorted(dur, key=lambda k: -sum(dur[k])):
            n = len(dur[k])
            us = sum(dur[k]) / n
            fe = ctr.get((k, "FETCH_SIZE"))
            wr = ctr.get((k, "WRITE_SIZE"))
            fmb = 2 * sum(fe) / len(fe) / 1e3 if fe else float("nan")  # KB -> MB, x2 gfx950
            wmb = sum(wr) / len(wr) / 1e3 if wr else float("nan")
            print("%-44s %7d %9.1f %10.1f %10.1f %8.0f" % (k[:44], n, us, fmb, wmb,
                                                          (fmb + wmb) / us * 1e3))


if __name__ == "__main__":
    main()
