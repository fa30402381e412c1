"""Run one term-pair conv config repeatedly (for PMC collection / A-B timing).

    python tools/conv_probe.py --layer 6 --config 1 --split 1 --iters 50
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "term-quantization_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import tq_native  # noqa: E402
import tq_ops  # noqa: E402
import tr_layer  # noqa: E402
from microbench import RESNET18_TR, make_layer, time_fn  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layer", type=int, default=6)
    ap.add_argument("--config", type=int, default=0)
    ap.add_argument("--split", type=int, default=0)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--codes", type=int, default=0, help="next-layer code outputs (0-2)")
    ap.add_argument("--residual", action="store_true", help="fp32 residual input")
    ap.add_argument("--no-out", action="store_true", help="no fp32 output (codes only)")
    ap.add_argument("--shape", default=None, help="cin,cout,k,stride,hin instead of --layer")
    ap.add_argument("--no-relu", action="store_true", help="no activation (signed codes)")
    ap.add_argument("--nonneg", action="store_true",
                    help="exactness windows for non-negative codes (the fused executor's)")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    cin, cout, k, s, hin = (RESNET18_TR[args.layer - 1] if args.shape is None else
                            tuple(int(v) for v in args.shape.split(",")))
    args.kc = None
    layer = make_layer(cin, cout, k, s, dev, args)
    cp = tq_ops.act_channels(cin)
    xi = torch.relu(torch.randn(args.batch, cin, hin, hin, device=dev)).to(
        memory_format=torch.channels_last)
    codes = torch.empty((args.batch, hin, hin, cp), dtype=layer.w_codes.dtype, device=dev)
    tq_native.act_encode(xi, True, 0.02, 9, 3, codes)
    ho = (hin + 2 * (k // 2) - k) // s + 1
    o = torch.empty((args.batch, cout, ho, ho), device=dev, memory_format=torch.channels_last)
    ws = tq_native.conv2d_workspace(args.batch * ho * ho, cout, dev)
    sc = torch.full((cout,), 1e-4, dtype=torch.float64, device=dev)
    sh = torch.zeros(cout, dtype=torch.float64, device=dev)
    res = torch.randn_like(o) if args.residual else None
    cpo = tq_ops.act_channels(cout)
    ca = torch.empty((args.batch, ho, ho, cpo), dtype=codes.dtype, device=dev) \
        if args.codes >= 1 else None
    cb = torch.empty_like(ca) if args.codes >= 2 else None
    q = (0.05, 9, 3)
    fn = lambda: tq_native.conv2d_termpair_fused(
        codes, layer.w_codes, cout, k, k, (s, s), (k // 2, k // 2), (1, 1), ho, ho,
        out=None if args.no_out else o, ch_scale=sc, ch_shift=sh, residual=res, relu=not args.no_relu,
        codes_a=ca, quant_a=q if ca is not None else None, codes_b=cb,
        quant_b=q if cb is not None else None,
        workspace=None if layer.engine == "mfma" else ws,
        split_k=args.split, config=args.config,
        kc_steps=layer.kc_steps_nonneg if args.nonneg else layer.kc_steps,
        kc_chunk=getattr(layer, "kc_chunk_nonneg" if args.nonneg else "kc_chunk", -1))
    t = time_fn(fn, args.iters)
    mac = args.batch * cout * ho * ho * cin * k * k
    print("layer %d cfg %d split %d: %.1f us  %.1f TMAC/s" % (args.layer, args.config,
                                                             args.split, t * 1e6,
                                                             mac / t / 1e12))


if __name__ == "__main__":
    main()
