"""Time the reference's own CPU encoder, bit_utils.hese (/root/reference/bit_utils.py:10-44),
in the build container -- a stated side baseline beside BENCH's C1, which times the oracle's
restatement oracle.hese_py (the reference Python never travels to the GPU box, so bench.py
cannot time it there).

Same sample as C1: 200,000 random q in [-511, 511] (numpy seed 0), one core, the encoder
called once per value as the reference's callers do (tr_layer.py / bit_utils.hese_bits).
Also times oracle.hese_py on the same values here, so the two are on one host.

    python -B tools/ref/time_ref_hese.py > profiles/r06_ref_hese_cpu.txt
"""
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, "/root/reference")
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import bit_utils  # noqa: E402  (the reference module; imports torch)
import oracle  # noqa: E402


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def best_of(fn, vals, reps=3):
    best = float("inf")
    for _ in range(reps):
        t0 = time.perf_counter()
        for q in vals:
            fn(q)
        best = min(best, time.perf_counter() - t0)
    return best


def main():
    rng = np.random.default_rng(0)
    vals = [int(v) for v in rng.integers(-511, 512, size=200000)]
    # the two encoders agree on the sample (their term lists as signed powers of two)
    for q in vals[:20000]:
        assert sorted(bit_utils.hese(q)) == sorted(oracle.hese_py(q)), q
    t_ref = best_of(bit_utils.hese, vals)
    t_py = best_of(oracle.hese_py, vals)
    print("host: %s, %d logical CPUs, python %s; one core" % (cpu_model(), os.cpu_count(),
                                                             platform.python_version()))
    print("sample: 200000 random q in [-511, 511] (numpy default_rng(0)), best of 3")
    print("reference bit_utils.hese (bit_utils.py:10-44): %.4f s = %.4g values/s" %
          (t_ref, len(vals) / t_ref))
    print("oracle.hese_py (restatement, BENCH C1):        %.4f s = %.4g values/s" %
          (t_py, len(vals) / t_py))
    print("ratio restatement / reference: %.2fx" % (t_ref / t_py))


if __name__ == "__main__":
    main()
