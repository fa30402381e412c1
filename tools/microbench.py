"""Kernel microbenchmarks on one GPU: the TR op (D1) and each ResNet-18 TR conv at batch 256.

    python tools/microbench.py [--batch 256] [--iters 20]

Prints one line per kernel: average time (HIP events on the launch stream), achieved
algorithmic GB/s (TR op, 8 B/elem; act encode, 6 B/elem) or term-sum MAC/s (conv)."""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "term-quantization_amd"))

import tq_native  # noqa: E402
import tq_ops  # noqa: E402
import tr_layer  # noqa: E402

# (cin, cout, k, stride, hin) of the 19 ResNet-18 TR convs
RESNET18_TR = [(64, 64, 3, 1, 56)] * 4 + [(64, 128, 3, 2, 56), (128, 128, 3, 1, 28),
                                          (64, 128, 1, 2, 56)] + \
    [(128, 128, 3, 1, 28)] * 2 + [(128, 256, 3, 2, 28), (256, 256, 3, 1, 14),
                                  (128, 256, 1, 2, 28)] + \
    [(256, 256, 3, 1, 14)] * 2 + [(256, 512, 3, 2, 14), (512, 512, 3, 1, 7),
                                  (256, 512, 1, 2, 14)] + [(512, 512, 3, 1, 7)] * 2


def time_fn(fn, iters, warmup=3):
    for _ in range(warmup):
        fn()
    s = torch.cuda.current_stream()
    start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    start.record(s)
    for _ in range(iters):
        fn()
    end.record(s)
    torch.cuda.synchronize()
    return start.elapsed_time(end) / iters * 1e-3


def make_layer(cin, cout, k, s, dev, args):
    """A ResNet-18 TR conv as the bench builds it (Kaiming-normal fan_out init)."""
    conv = torch.nn.Conv2d(cin, cout, k, s, k // 2, bias=False)
    torch.nn.init.kaiming_normal_(conv.weight, mode="fan_out", nonlinearity="relu")
    layer = tr_layer.TRConv2dLayer(conv.to(dev), 9, 3, 9, 8, 12)
    if args.kc is not None and layer.engine == "mfma":
        layer.kc_steps = args.kc  # timing only: results may be inexact
    return layer


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--engine", choices=("mfma", "valu"), default="mfma")
    ap.add_argument("--kc", type=int, default=None,
                    help="timing only: override the MFMA flush interval (0 = no flush)")
    ap.add_argument("--sweep", action="store_true",
                    help="time every tile config x K-split per layer (fused NHWC entry)")
    args = ap.parse_args()
    os.environ["TQ_CONV_ENGINE"] = args.engine
    dev = torch.device("cuda:0")
    torch.manual_seed(0)

    x = torch.relu(torch.randn(256, 64, 56, 56, device=dev))
    flat = x.view(1, -1, 1, 1)
    out = torch.empty_like(flat)
    t = time_fn(lambda: tq_native.tr_into(flat, out, 0.05, 9, 1, 3), args.iters)
    n = flat.numel()
    print("tr_op D1 g=1: %.1f us  %.0f GB/s (8 B/elem)  %.3f Telem/s" % (
        t * 1e6, 8 * n / t / 1e9, n / t / 1e12))

    xl = x.to(memory_format=torch.channels_last)
    codes = torch.empty((256, 56, 56, 64), dtype=torch.int16, device=dev)
    t = time_fn(lambda: tq_native.act_encode(xl, True, 0.05, 9, 3, codes), args.iters)
    print("act_encode NHWC: %.1f us  %.0f GB/s (6 B/elem)" % (t * 1e6, 6 * n / t / 1e9))

    w = torch.randn(512, 512, 3, 3, device=dev) * 0.05
    t = time_fn(lambda: tr_layer.tr_cuda.tr(w, w.abs().max().item() / 256, 9, 8, 12), 5)
    print("tr_op weight 512x512x3x3 g=8 k=12: %.1f us" % (t * 1e6))

    total_mac, total_t = 0, 0.0
    for i, (cin, cout, k, s, hin) in enumerate(RESNET18_TR):
        layer = make_layer(cin, cout, k, s, dev, args)
        layer.input_quant.tracking = False
        layer.input_quant.sf = 0.02
        xi = torch.relu(torch.randn(args.batch, cin, hin, hin, device=dev)).to(
            memory_format=torch.channels_last)
        ho = (hin + 2 * (k // 2) - k) // s + 1
        cp = tq_ops.act_channels(cin)
        codes = torch.empty((args.batch, hin, hin, cp), dtype=layer.w_codes.dtype, device=dev)
        tq_native.act_encode(xi, True, 0.02, 9, 3, codes)
        o = torch.empty((args.batch, cout, ho, ho), device=dev,
                        memory_format=torch.channels_last)
        fn = lambda: tq_native.conv2d_termpair(codes, layer.w_codes, cout, k, k, (s, s),
                                               (k // 2, k // 2), (1, 1), 1e-4, None, o, True,
                                               layer.kc_steps)
        t = time_fn(fn, args.iters)
        mac = args.batch * cout * ho * ho * cin * k * k
        total_mac += mac
        total_t += t
        print("conv%02d %3d->%3d k%d s%d %2dx%2d: %8.1f us  %6.1f TMAC/s  kc=%d" % (
            i + 1, cin, cout, k, s, hin, hin, t * 1e6, mac / t / 1e12, layer.kc_steps))
    print("conv total: %.2f ms  %.1f TMAC/s  -> %.0f img/s (convs only)" % (
        total_t * 1e3, total_mac / total_t / 1e12, args.batch / total_t))
    if args.sweep:
        sweep(args, dev)


def sweep(args, dev):
    mfma = args.engine == "mfma"
    ncfg = (tq_native.lib().tq_conv2d_mfma_num_configs() if mfma else
            tq_native.lib().tq_conv2d_num_configs())
    best_total = 0.0
    auto_total = 0.0
    seen = {}
    for i, (cin, cout, k, s, hin) in enumerate(RESNET18_TR):
        key = (cin, cout, k, s, hin)
        if key in seen:
            best_total += seen[key][0]
            auto_total += seen[key][1]
            continue
        layer = make_layer(cin, cout, k, s, dev, args)
        cp = tq_ops.act_channels(cin)
        xi = torch.relu(torch.randn(args.batch, cin, hin, hin, device=dev)).to(
            memory_format=torch.channels_last)
        codes = torch.empty((args.batch, hin, hin, cp), dtype=layer.w_codes.dtype, device=dev)
        tq_native.act_encode(xi, True, 0.02, 9, 3, codes)
        ho = (hin + 2 * (k // 2) - k) // s + 1
        o = torch.empty((args.batch, cout, ho, ho), device=dev,
                        memory_format=torch.channels_last)
        ws = tq_native.conv2d_workspace(args.batch * ho * ho, cout, dev)
        sc = torch.full((cout,), 1e-4, dtype=torch.float64, device=dev)
        sh = torch.zeros(cout, dtype=torch.float64, device=dev)
        mac = args.batch * cout * ho * ho * cin * k * k
        # the bench's heavier epilogue: ReLU, fp32 output and next-layer codes
        ca = torch.empty((args.batch, ho, ho, tq_ops.act_channels(cout)),
                         dtype=layer.w_codes.dtype, device=dev)
        res = {}
        for cfg in range(0, ncfg + 1):
            for sp in ([1, -1, 3] if cfg and not mfma else [0]):
                fn = lambda: tq_native.conv2d_termpair_fused(
                    codes, layer.w_codes, cout, k, k, (s, s), (k // 2, k // 2), (1, 1), ho, ho,
                    out=o, ch_scale=sc, ch_shift=sh, relu=True, codes_a=ca,
                    quant_a=(0.05, 9, 3), workspace=None if mfma else ws,
                    split_k=sp, config=cfg, kc_steps=layer.kc_steps_nonneg,
                    kc_chunk=layer.kc_chunk_nonneg)  # relu'd inputs, as the fused executor
                res[(cfg, sp)] = time_fn(fn, max(5, args.iters // 2))
        best = min(res, key=res.get)
        auto = res[(0, 0)]
        seen[key] = (res[best], auto)
        best_total += res[best]
        auto_total += auto
        line = " ".join("c%ds%d=%.0f" % (c, sp, t * 1e6) for (c, sp), t in sorted(res.items()))
        print("sweep conv%02d %s best=c%ds%d %.1f us (%.1f TMAC/s) auto %.1f us | %s" % (
            i + 1, key, best[0], best[1], res[best] * 1e6, mac / res[best] / 1e12, auto * 1e6,
            line))
    print("sweep totals: best %.2f ms, auto %.2f ms" % (best_total * 1e3, auto_total * 1e3))


if __name__ == "__main__":
    main()
