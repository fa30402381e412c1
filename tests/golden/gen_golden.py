"""Generate the golden fixtures under tests/golden/ from the reference itself.

Run in the build container only (it reads /root/reference, which does not exist on the GPU
box):  python -B tests/golden/gen_golden.py

What it produces (all plain data, no reference source):
  hese_bit_utils.npz         q in [-4096, 4096) -> (pos, neg) uint32 masks of the signed terms
                              returned by the reference CPU encoder bit_utils.hese
                              (bit_utils.py:10-44).
  hese_bit_utils_sha256.json SHA-256 of the (pos || neg) little-endian uint32 table for every
                              q in [0, 2^17) -- the full range of 16-bit quantized values and
                              one more bit, checked by tests/test_oracle.py without storing
                              512 KB of masks.
  tr_layer_hese_len.npz      q in [-4096, 4096) -> len(tr_layer.hese(q)) (tr_layer.py:9-41),
                              the per-weight term count behind compute_compressed_hese.  The
                              function is executed from the file's text (tr_layer.py builds a
                              CUDA extension at import time, so the module is not imported).
  published_results.json     the analytic counts and accuracies the reference publishes in
                              results/*.json (its only known answers).
"""
import ast
import hashlib
import json
import os
import sys

import numpy as np

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def masks_from_terms(terms):
    pos = neg = 0
    for t in terms:
        e = abs(t).bit_length() - 1
        assert abs(t) == 1 << e
        if t > 0:
            pos |= 1 << e
        else:
            neg |= 1 << e
    return pos, neg


def main():
    sys.dont_write_bytecode = True  # never write __pycache__ into the read-only reference
    sys.path.insert(0, REF)
    import bit_utils  # the reference's pure-Python HESE encoder

    qs = np.arange(-4096, 4096, dtype=np.int64)
    pos = np.zeros(qs.shape, np.uint32)
    neg = np.zeros(qs.shape, np.uint32)
    for i, q in enumerate(qs.tolist()):
        pos[i], neg[i] = masks_from_terms(bit_utils.hese(q))
    np.savez_compressed(os.path.join(OUT, "hese_bit_utils.npz"), q=qs, pos=pos, neg=neg)

    n = 1 << 17
    fp = np.zeros(n, np.uint32)
    fn = np.zeros(n, np.uint32)
    for q in range(n):
        fp[q], fn[q] = masks_from_terms(bit_utils.hese(q))
    digest = hashlib.sha256(fp.astype("<u4").tobytes() + fn.astype("<u4").tobytes()).hexdigest()
    with open(os.path.join(OUT, "hese_bit_utils_sha256.json"), "w") as f:
        json.dump({"q_range": [0, n], "layout": "pos[0:n] || neg[0:n], uint32 little-endian",
                   "sha256": digest, "source": "bit_utils.hese (bit_utils.py:10-44)"}, f,
                  indent=1)

    # tr_layer.hese: executed from the file text, module-level code (the JIT build) skipped
    src = open(os.path.join(REF, "tr_layer.py")).read()
    tree = ast.parse(src)
    fdef = [nd for nd in tree.body if isinstance(nd, ast.FunctionDef) and nd.name == "hese"][0]
    ns = {}
    exec(compile(ast.Module(body=[fdef], type_ignores=[]), "tr_layer.py", "exec"), ns)
    lens = np.array([len(ns["hese"](q)) for q in qs.tolist()], np.int32)
    np.savez_compressed(os.path.join(OUT, "tr_layer_hese_len.npz"), q=qs, length=lens)

    published = {}
    for name in sorted(os.listdir(os.path.join(REF, "results"))):
        if name.endswith(".json"):
            with open(os.path.join(REF, "results", name)) as f:
                published[name] = json.load(f)
    with open(os.path.join(OUT, "published_results.json"), "w") as f:
        json.dump(published, f, indent=1, sort_keys=True)
    print("golden fixtures written to", OUT, "sha256", digest)


if __name__ == "__main__":
    main()
