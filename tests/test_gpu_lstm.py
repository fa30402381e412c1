"""LSTM-650 TQ on the GPU (BASELINE configs[2]; evaluate_lstm.py:139-151, tr_layer.py:162-201):
RNNModel(33278, 650, 650, 2, tied) converted with g=8, k=12, wb=db=dt=8, calibrated on
synthetic token ids, then one 35 x 10 chunk.

  * the TR'd weight_ih_l0 / weight_hh_l0 (650 % 8 != 0: partial last group) and
    decoder weight are bit-exact oracle.tr() of the original weights;
  * the shared quantizer's outputs on emb, h0 and c0 are bit-exact oracle.tr() (g = 1);
  * the log-probs are within 1e-5 of an fp64 CPU composition of the oracle-TR'd tensors
    (fp64 LSTM on TR(emb), TR(h0), TR(c0) with the TR'd layer-0 weights, decoder on the
    unquantized LSTM output as the reference's TRLinearLayer does, log_softmax).
Both TRLSTMLayer paths: the reference composition (MIOpen LSTM) and ``termpair=True`` (layer
0's input projection and first recurrent step as exact term-pair GEMMs, tq_lstm_cell_f32)."""
import pytest
import torch
import torch.nn as nn

import oracle
import tr_layer

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
VOCAB, NHID, BPTT, BSZ = 33278, 650, 35, 10


def _oracle_w(w, bits, g, k):
    sf = w.abs().max().item() / 2 ** (bits - 1)
    return torch.from_numpy(oracle.tr(w.detach().cpu().contiguous().numpy(), sf, bits, g, k))


@pytest.mark.parametrize("termpair,seq", [(False, None), (True, "1"), (True, "layer"),
                                          (True, "0"), (True, "miopen")])
def test_lstm650_tq_chunk_against_oracle(termpair, seq, monkeypatch):
    """seq (term-pair path): "1" (default) = both layers in wavefront order, T + 1 launches
    (tq_lstm_seq2_f32), "layer" = each layer's recurrence from one call (tq_lstm_seq_f32,
    TQ_LSTM_WAVE=0), "0" = per-step launches (a GEMM + tq_lstm_cell_f32 per step, MIOpen for
    layer 1), "miopen" = the one-call recurrence for layer 0, MIOpen above."""
    import evaluate_lstm
    import tq_native
    if seq == "miopen":
        monkeypatch.setenv("TQ_LSTM_UPPER", "miopen")
    elif seq == "layer":
        monkeypatch.setenv("TQ_LSTM_WAVE", "0")
    elif seq is not None:
        monkeypatch.setenv("TQ_LSTM_SEQ", seq)
    tq_native.sync_faults()
    from lstm_models.model import RNNModel
    torch.manual_seed(1111)
    model = RNNModel("LSTM", VOCAB, NHID, NHID, 2, 0.5, True).to(DEV).eval()
    w_ih = model.rnn.weight_ih_l0.detach().clone()
    w_hh = model.rnn.weight_hh_l0.detach().clone()
    w_dec = model.decoder.weight.detach().clone()
    st = evaluate_lstm.static_lstm_layer_settings(model, 8, 8, 12)
    q = evaluate_lstm.convert_model(model, st, 8, 8, termpair=termpair).eval()
    lstm = q.rnn
    assert isinstance(lstm, tr_layer.TRLSTMLayer)
    assert lstm.termpair == termpair
    assert isinstance(q.decoder, tr_layer.TRLinearLayer)
    # weights: bit-exact, including the partial last group of every 650-wide row
    assert torch.equal(lstm.lstm.weight_ih_l0.detach().cpu(), _oracle_w(w_ih, 8, 8, 12))
    assert torch.equal(lstm.lstm.weight_hh_l0.detach().cpu(), _oracle_w(w_hh, 8, 8, 12))
    wq_dec = _oracle_w(w_dec, 8, 8, 12)
    assert torch.equal(q.decoder.linear.weight.detach().cpu(), wq_dec)

    # calibration on synthetic token ids (evaluate_lstm.py:146-147), then one chunk
    g = torch.Generator().manual_seed(7)
    calib = evaluate_lstm.batchify(torch.randint(0, VOCAB, (BPTT * BSZ * 2 + BSZ,), generator=g),
                                   BSZ, DEV)
    crit = nn.NLLLoss()
    evaluate_lstm.evaluate(q, calib, VOCAB, BSZ, BPTT, crit)
    tr_layer.set_tr_tracking(q, False)
    sf = lstm.input_quant.sf
    assert sf > 0
    data = torch.randint(0, VOCAB, (BPTT, BSZ), generator=g).to(DEV)
    with torch.no_grad():
        hidden = (torch.randn(2, BSZ, NHID, generator=g).to(DEV) * 0.3,
                  torch.randn(2, BSZ, NHID, generator=g).to(DEV) * 0.3)
        seen = []
        h = lstm.input_quant.register_forward_hook(lambda m, i, o: seen.append((i[0], o)))
        try:
            logp, (hn, cn) = q(data, hidden)
        finally:
            h.remove()
    torch.cuda.synchronize()
    # the shared quantizer ran on emb, h0, c0 (tr_layer.py:191-193): bit-exact (the term-pair
    # path encodes emb inside its term-pair GEMM: its quantizer call sees h0 and c0 only)
    if termpair:
        seen.insert(0, (q.encoder(data), tr_layer.tr_cuda.tr(
            q.encoder(data).contiguous().view(1, -1, 1, 1), sf, 8, 1, 8).view(BPTT, BSZ, NHID)))
    assert len(seen) == 3
    for x, y in seen:
        exp = oracle.tr(x.detach().cpu().contiguous().numpy().reshape(1, -1, 1, 1), sf, 8, 1, 8)
        assert torch.equal(y.detach().cpu(), torch.from_numpy(exp).view(y.shape))
    embq, h0q, c0q = (y.detach().cpu().double() for _, y in seen)

    # fp64 composition on the CPU from the oracle-TR'd tensors
    ref = nn.LSTM(NHID, NHID, 2).double()
    with torch.no_grad():
        ref.weight_ih_l0.copy_(_oracle_w(w_ih, 8, 8, 12).double())
        ref.weight_hh_l0.copy_(_oracle_w(w_hh, 8, 8, 12).double())
        for name in ("bias_ih_l0", "bias_hh_l0", "weight_ih_l1", "weight_hh_l1", "bias_ih_l1",
                     "bias_hh_l1"):
            getattr(ref, name).copy_(getattr(lstm.lstm, name).detach().cpu().double())
        out, (hr, cr) = ref(embq, (h0q, c0q))
        dec = out @ wq_dec.double().t() + \
            q.decoder.linear.bias.detach().cpu().double()
        lp_ref = torch.log_softmax(dec.view(-1, VOCAB), dim=1)
        lse = torch.logsumexp(dec.view(-1, VOCAB), dim=1, keepdim=True)
    lp = logp.detach().cpu().double()
    err = (lp - lp_ref).abs()
    # per element: lp = dec - lse, each term carrying fp32 rounding relative to its own size
    mag = dec.view(-1, VOCAB).abs() + lse.abs()
    ratio = err / (1e-5 * mag)
    assert bool((ratio <= 1.0).all()), float(ratio.max())
    assert float((hn.cpu().double() - hr).abs().max()) <= 1e-5
    assert float((cn.cpu().double() - cr).abs().max()) <= 1e-5 * max(1.0, float(cr.abs().max()))
