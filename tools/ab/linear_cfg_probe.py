"""Per-config time of the term-pair GEMM behind the LSTM-650 layer-0 input projection
(tr_linear: 350 rows = bptt 35 x batch 10, 650 -> 2600, a 1x1 term-pair conv on the MFMA
engine) with random small codes; config 0 = the engine's default choice.
python tools/ab/linear_cfg_probe.py"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "term-quantization_amd"))
import tq_native  # noqa: E402
import tq_ops  # noqa: E402

dev = torch.device("cuda:0")
M, C, O = 350, 650, 2600
torch.manual_seed(0)
wq = torch.randint(-3, 4, (O, C, 1, 1), dtype=torch.int32)
packed, cp = tq_ops.pack_conv_weight(wq, "mfma")
packed = packed.to(dev)
codes = torch.randint(-3, 4, (M, 1, 1, cp), dtype=torch.int16).to(torch.float16).to(dev)
codes[..., C:] = 0
out = torch.empty((M, O, 1, 1), device=dev).contiguous(memory_format=torch.channels_last)
sc = torch.ones(O, device=dev)
sh = torch.zeros(O, device=dev)
ref = None
for cfg in range(0, tq_native.lib().tq_conv2d_mfma_num_configs() + 1):
    try:
        def run():
            tq_native.conv2d_termpair_fused(codes, packed, O, 1, 1, (1, 1), (0, 0), (1, 1), 1,
                                            1, out=out, ch_scale=sc, ch_shift=sh, config=cfg)
        run()
        torch.cuda.synchronize()
    except Exception as e:  # noqa: BLE001
        print("config %2d: %s" % (cfg, str(e)[:60]))
        continue
    same = ref is None or torch.equal(out, ref)
    if ref is None:
        ref = out.clone()
    for _ in range(3):
        run()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        run()
    e1.record()
    torch.cuda.synchronize()
    print("config %2d: %.1f us per launch%s" % (cfg, e0.elapsed_time(e1) / 50 * 1e3,
                                               "" if same else "  (DIFFERENT RESULT)"))
