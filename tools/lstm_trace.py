"""LSTM-650 TQ chunk (batch 10 x bptt 35) for a kernel trace: python tools/lstm_trace.py
[--termpair 0|1] [--chunks N].  Run under rocprofv3 --kernel-trace --stats; prints the
host-timed ms per chunk."""
import argparse
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "term-quantization_amd"))
import evaluate_lstm  # noqa: E402
import tr_layer  # noqa: E402
from lstm_models import model as model_mod  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--termpair", type=int, default=1)
    ap.add_argument("--chunks", type=int, default=20)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.manual_seed(1111)
    ntokens, bsz, bptt = evaluate_lstm.WT2_VOCAB, 10, 35
    model = model_mod.RNNModel("LSTM", ntokens, 650, 650, 2, 0.5, True).to(dev).eval()
    st = evaluate_lstm.static_lstm_layer_settings(model, 8, 8, 12)
    q = evaluate_lstm.convert_model(model, st, 8, 8, termpair=bool(args.termpair)).eval()
    data = evaluate_lstm.batchify(torch.randint(0, ntokens, (bptt * bsz * 4 + bsz,)), bsz, dev)
    x = evaluate_lstm.get_batch(data, 0, bptt)[0]
    with torch.no_grad():
        q(x, model.init_hidden(bsz))
        tr_layer.set_tr_tracking(q, False)
        hidden = model.init_hidden(bsz)
        for _ in range(3):
            q(x, hidden)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.chunks):
            q(x, hidden)
        torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.chunks
    print("termpair=%d: %.3f ms per chunk, %.0f tokens/s" % (args.termpair, dt * 1e3,
                                                            bptt * bsz / dt))


if __name__ == "__main__":
    main()
