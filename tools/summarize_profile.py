"""Turn a tools/gpu_profile.sh run (gpurun_out/<tag>/) into committed profile summaries.

    python tools/summarize_profile.py <tag>

Writes profiles/<tag>_kernel_stats.csv (rocprofv3 --kernel-trace --stats, verbatim),
profiles/<tag>_summary.json (per-kernel average duration and per-launch HBM bytes) and
refreshes profiles/pmc_traffic.json (read by bench.py for roofline.traffic).

HBM bytes per launch follow MI355X_MICROARCH.md "HBM": FETCH_SIZE and WRITE_SIZE come from
separate --pmc passes, both in KiB; on gfx950 FETCH_SIZE counts half the bytes of a wide
(16 B/lane) coalesced read (global_load and LDS-DMA alike), so it is doubled for the TQ
kernels (all of whose global loads are 16-byte vectors); WRITE_SIZE is exact for 16-byte
stores.
"""
import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNELS = {  # summary key -> kernel-name substrings (every MFMA term-pair conv engine)
    "conv2d_tp": ("conv2d_tp_kernel",),
    "conv2d_tp_mfma": ("conv2d_tp_mfma", "conv2d_tp_patch", "conv2d_tp_direct",
                       "conv2d_tp_strip", "conv2d_tp_ring", "conv2d_tp_pw", "conv2d_tp_c64",
                       "conv2d_tp_xp"),
    "act_encode": ("act_encode_kernel",),
    "stem_pool_encode": ("bn_relu_maxpool_encode_kernel",),
    "stem_conv_pool": ("stem_conv_pool_kernel",),
    "tr_elem": ("tr_elem_kernel",),
    "tr_group": ("tr_group_kernel",),
}


def pmc(path, counter):
    per = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            per[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return per


def busy_us(trace_csv, needles):
    """Union of the launch intervals of the matching kernels (us): the GPU time during which
    at least one of them runs; equals the summed durations when launches do not overlap
    (one stream) and is shorter when bench.py's chunk streams overlap them."""
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
                for r in csv.DictReader(open(trace_csv))
                if any(nd in r["Kernel_Name"] for nd in needles))
    busy, cs, ce = 0, None, None
    for s, e in iv:
        if ce is None or s > ce:
            if ce is not None:
                busy += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    if ce is not None:
        busy += ce - cs
    return busy / 1e3


def main(tag):
    src = os.path.join(ROOT, "gpurun_out", tag)
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)
    stats_csv = os.path.join(src, "kt", "kt_kernel_stats.csv")
    shutil.copy(stats_csv, os.path.join(dst, "%s_kernel_stats.csv" % tag))
    stats = {r["Name"]: r for r in csv.DictReader(open(stats_csv))}
    fetch = pmc(os.path.join(src, "pmc_FETCH_SIZE", "pmc_counter_collection.csv"), "FETCH_SIZE")
    write = pmc(os.path.join(src, "pmc_WRITE_SIZE", "pmc_counter_collection.csv"), "WRITE_SIZE")
    summary = {"tag": tag, "kernels": {}}
    for key, needles in KERNELS.items():
        names = [n for n in stats if any(nd in n for nd in needles)]
        if not names:
            continue
        calls = sum(int(stats[n]["Calls"]) for n in names)
        total_ns = sum(float(stats[n]["TotalDurationNs"]) for n in names)
        f = [v for n in fetch if any(nd in n for nd in needles) for v in fetch[n]]
        w = [v for n in write if any(nd in n for nd in needles) for v in write[n]]
        entry = {"variants": names, "calls": calls, "avg_duration_us": total_ns / calls / 1e3}
        trace_csv = os.path.join(src, "kt", "kt_kernel_trace.csv")
        if os.path.exists(trace_csv):
            entry["busy_us_per_launch"] = busy_us(trace_csv, needles) / calls
        if f and w:
            entry["fetch_bytes_per_launch"] = 2.0 * sum(f) / len(f) * 1024
            entry["write_bytes_per_launch"] = sum(w) / len(w) * 1024
            entry["hbm_bytes_per_launch"] = (entry["fetch_bytes_per_launch"] +
                                             entry["write_bytes_per_launch"])
        summary["kernels"][key] = entry
    bench = os.path.join(src, "bench.json")
    if os.path.exists(bench):
        summary["bench"] = json.loads(open(bench).read().strip().splitlines()[-1])
    with open(os.path.join(dst, "%s_summary.json" % tag), "w") as fp:
        json.dump(summary, fp, indent=1)
    conv = summary["kernels"].get("conv2d_tp", {})
    conv_m = summary["kernels"].get("conv2d_tp_mfma", {})
    enc = summary["kernels"].get("act_encode", {})
    stem = summary["kernels"].get("stem_pool_encode", {})
    stem_conv = summary["kernels"].get("stem_conv_pool", {})
    with open(os.path.join(dst, "pmc_traffic.json"), "w") as fp:
        json.dump({"source": "profiles/%s_summary.json" % tag,
                   "conv2d_tp_bytes_per_launch": conv.get("hbm_bytes_per_launch"),
                   "conv2d_tp_mfma_bytes_per_launch": conv_m.get("hbm_bytes_per_launch"),
                   "act_encode_bytes_per_launch": enc.get("hbm_bytes_per_launch"),
                   "stem_pool_encode_bytes_per_launch": stem.get("hbm_bytes_per_launch"),
                   "stem_conv_pool_bytes_per_launch": stem_conv.get("hbm_bytes_per_launch")}, fp,
                  indent=1)
    for k, v in summary["kernels"].items():
        print(k, {a: b for a, b in v.items() if a != "variants"})


if __name__ == "__main__":
    main(sys.argv[1])
