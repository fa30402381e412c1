"""LSTM-650 WikiText-2 UQ/TQ sweep -- the reference's evaluate_lstm.py
(evaluate_lstm.py:1-176), same CLI and result JSON (ppls, tmacs, param_bits).

    python evaluate_lstm.py --wb 8 --wt 12 --db 8 --dt 8 --gs 8 --out-file r.json
    python evaluate_lstm.py --synthetic ...   # random-init 2x650 LSTM, random token ids

Offline notes: the reference loads a pickled whole model (torch.load of
pretrained_models/lstm.pt) -- here ``--checkpoint`` takes a state_dict loaded weights-only;
the WikiText-2 train split (needed for the vocabulary) is absent, so ``--synthetic`` draws
token ids uniformly from the 33,278-word vocabulary.
"""
import argparse
import json
import math
from copy import deepcopy

import torch
import torch.nn as nn

import lstm_models.model as model_mod
import profile_model
from tr_layer import TRLinearLayer, TRLSTMLayer, set_tr_tracking

WT2_VOCAB = 33278


def replace_lstm_layers(model, tr_params, data_bits, data_terms, termpair=True):
    """``termpair`` (an addition): TRLSTMLayer's term-pair layer-0 path (tr_layer.py; False =
    the library LSTM on the TR'd tensors, the reference's literal composition)."""
    curr_layer = 0
    for name, layer in list(model.named_modules()):
        if isinstance(layer, (nn.Linear, nn.LSTM)):
            module_keys = name.split('.')
            module = model
            for k in module_keys[:-1]:
                module = module._modules[k]

            weight_bits, group_size, weight_terms = tr_params[curr_layer]
            if isinstance(layer, nn.LSTM):
                layer = TRLSTMLayer(layer, data_bits, data_terms, weight_bits,
                                    group_size, weight_terms, termpair=termpair)
            elif isinstance(layer, nn.Linear):
                layer = TRLinearLayer(layer, data_bits, data_terms, weight_bits,
                                      group_size, weight_terms)

            module._modules[module_keys[-1]] = layer
            curr_layer += 1

    return model


def static_lstm_layer_settings(model, weight_bits, group_size, num_terms):
    stats = []
    for _, layer in model.named_modules():
        if isinstance(layer, (nn.Linear, nn.LSTM)):
            stats.append((weight_bits, group_size, num_terms))
    return stats


def convert_model(model, tr_params, data_bits, data_terms, termpair=True):
    model = deepcopy(model)
    return replace_lstm_layers(model, tr_params, data_bits, data_terms, termpair)


def batchify(data, bsz, device):
    nbatch = data.size(0) // bsz
    data = data.narrow(0, 0, nbatch * bsz)
    return data.view(bsz, -1).t().contiguous().to(device)


def repackage_hidden(h):
    if isinstance(h, torch.Tensor):
        return h.detach()
    return tuple(repackage_hidden(v) for v in h)


def get_batch(source, i, bptt):
    seq_len = min(bptt, len(source) - 1 - i)
    data = source[i:i + seq_len]
    target = source[i + 1:i + 1 + seq_len].view(-1)
    return data, target


def evaluate(model, data_source, ntokens, eval_batch_size, bptt, criterion):
    model.eval()
    total_loss = 0.
    hidden = model.init_hidden(eval_batch_size)
    with torch.no_grad():
        for i in range(0, data_source.size(0) - 1, bptt):
            data, targets = get_batch(data_source, i, bptt)
            output, hidden = model(data, hidden)
            hidden = repackage_hidden(hidden)
            total_loss += len(data) * criterion(output, targets).item()
    return total_loss / (len(data_source) - 1)


def main(argv=None):
    parser = argparse.ArgumentParser(description='PyTorch Wikitext-2 LSTM Language Model')
    parser.add_argument('--data', type=str, default='./lstm_models/data/wikitext-2/')
    parser.add_argument('--model', type=str, default='LSTM')
    parser.add_argument('--emsize', type=int, default=650)
    parser.add_argument('--nhid', type=int, default=650)
    parser.add_argument('--nlayers', type=int, default=2)
    parser.add_argument('--dropout', type=float, default=0.5)
    parser.add_argument('--tied', action='store_false')
    parser.add_argument('--seed', type=int, default=1111)
    parser.add_argument('--cuda', action='store_false')
    parser.add_argument('--bptt', type=int, default=35)
    parser.add_argument('--wb', nargs='+', type=int, help='weight bits')
    parser.add_argument('--wt', nargs='+', type=int, help='weight terms')
    parser.add_argument('--db', nargs='+', type=int, help='data bits')
    parser.add_argument('--dt', nargs='+', type=int, help='data terms')
    parser.add_argument('--gs', nargs='+', type=int, help='group sizes')
    parser.add_argument('--out-file', help='Output file')
    parser.add_argument('--synthetic', action='store_true',
                        help='random-init model and uniform random token ids')
    parser.add_argument('--synthetic-tokens', type=int, default=35 * 10 * 8 + 10)
    parser.add_argument('--checkpoint', default='pretrained_models/lstm.pt',
                        help='RNNModel state_dict (weights-only load)')
    args = parser.parse_args(argv)

    device = torch.device("cuda" if args.cuda else "cpu")
    torch.manual_seed(args.seed)
    eval_batch_size = 10
    if args.synthetic:
        ntokens = WT2_VOCAB
        test_tokens = torch.randint(0, ntokens, (args.synthetic_tokens,))
    else:
        import lstm_models.data as data
        corpus = data.Corpus(args.data)
        ntokens = len(corpus.dictionary)
        test_tokens = corpus.test
    test_data = batchify(test_tokens, eval_batch_size, device)
    model = model_mod.RNNModel(args.model, ntokens, args.emsize, args.nhid, args.nlayers,
                               args.dropout, args.tied)
    if not args.synthetic:
        model.load_state_dict(torch.load(args.checkpoint, map_location='cpu',
                                         weights_only=True))
    model = model.to(device)
    criterion = nn.NLLLoss()

    settings = zip(args.wb, args.wt, args.db, args.dt, args.gs)
    results = {'ppls': [], 'tmacs': [], 'param_bits': []}
    for wb, wt, db, dt, gs in settings:
        tr_params = static_lstm_layer_settings(model, wb, gs, wt)
        qmodel = convert_model(model, tr_params, db, dt)

        evaluate(qmodel, test_data, ntokens, eval_batch_size, args.bptt, criterion)
        set_tr_tracking(qmodel, False)
        test_loss = evaluate(qmodel, test_data, ntokens, eval_batch_size, args.bptt, criterion)
        inputs = (get_batch(test_data, 0, args.bptt)[0], model.init_hidden(eval_batch_size))
        tmacs, param_bits = profile_model.get_model_ops(qmodel, inputs=inputs)
        ppl = math.exp(test_loss)
        results['ppls'].append(ppl)
        results['tmacs'].append(tmacs)
        results['param_bits'].append(param_bits)
        print(wb, wt, db, dt, gs, ppl, tmacs, param_bits)

    if args.out_file:
        with open(args.out_file, 'w') as fp:
            json.dump(results, fp)
    return results


if __name__ == '__main__':
    main()
