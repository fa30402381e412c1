"""MNIST MLP UQ/TQ sweep -- the reference's evaluate_mlp.py (evaluate_mlp.py:1-95).

    python evaluate_mlp.py --wb 4 4 --wt 6 12 --db 6 6 --dt 6 6 --gs 16 16 --out-file r.json
    python evaluate_mlp.py --synthetic ...      # random-init MLP + N(0,1) 1x28x28 images

Same CLI and result JSON (accs, tmacs, param_bits).  The reference's profiling call passes
``input_shape=`` to get_model_ops and crashes (evaluate_mlp.py:88 vs profile_model.py:51);
here it passes a 1x1x28x28 input as intended.  ``--no-cuda`` (BASELINE configs[0]) runs the
TR layers on CPU tensors through the host TR op (libtq_host.so, include/tq_host.h) -- the
reference's CPU run would fail there, since its extension rejects CPU tensors.
"""
import argparse
import json
from copy import deepcopy

import torch
import torch.nn as nn

import util
from profile_model import get_model_ops
from tr_layer import TRLinearLayer, set_tr_tracking
from train_mlp import MNISTMLP, test


def replace_linear_layers(model, tr_params, data_bits, data_terms):
    curr_layer = 0
    for name, layer in list(model.named_modules()):
        if isinstance(layer, nn.Linear):
            module_keys = name.split('.')
            module = model
            for k in module_keys[:-1]:
                module = module._modules[k]

            weight_bits, group_size, weight_terms = tr_params[curr_layer]
            layer = TRLinearLayer(layer, data_bits, data_terms, weight_bits,
                                  group_size, weight_terms)

            module._modules[module_keys[-1]] = layer
            curr_layer += 1

    return model


def static_linear_layer_settings(model, weight_bits, group_size, num_terms):
    stats = []
    for name, layer in model.named_modules():
        if isinstance(layer, nn.Linear):
            stats.append((weight_bits, group_size, num_terms))
    return stats


class SyntheticMNIST(object):
    """N(0,1) 1x28x28 images with random labels, DataLoader-like."""

    def __init__(self, num_samples=10000, batch_size=128, seed=0):
        self.loader = util.SyntheticImageNet(num_samples, batch_size, image_size=28, seed=seed)
        self.dataset = self.loader.dataset

    def __len__(self):
        return len(self.loader)

    def __iter__(self):
        for i in range(len(self.loader)):
            x, y = self.loader.batch(i)
            yield x[:, :1].contiguous(), y % 10


def main(argv=None):
    parser = argparse.ArgumentParser(description='PyTorch MNIST Example')
    parser.add_argument('--test-batch-size', type=int, default=128, metavar='N',
                        help='input batch size for testing (default: 128)')
    parser.add_argument('--no-cuda', action='store_true', default=False,
                        help='disables CUDA training')
    parser.add_argument('--wb', nargs='+', type=int, help='weight bits')
    parser.add_argument('--wt', nargs='+', type=int, help='weight terms')
    parser.add_argument('--db', nargs='+', type=int, help='data bits')
    parser.add_argument('--dt', nargs='+', type=int, help='data terms')
    parser.add_argument('--gs', nargs='+', type=int, help='group sizes')
    parser.add_argument('--out-file', help='Output file')
    parser.add_argument('--synthetic', action='store_true',
                        help='random-init MLP and N(0,1) images (no MNIST / checkpoint)')
    parser.add_argument('--checkpoint', default='pretrained_models/mnist_mlp.pt',
                        help='state_dict of MNISTMLP (loaded weights-only)')
    args = parser.parse_args(argv)
    use_cuda = not args.no_cuda and torch.cuda.is_available()
    device = torch.device("cuda" if use_cuda else "cpu")

    if args.synthetic:
        test_loader = SyntheticMNIST(batch_size=args.test_batch_size)
        torch.manual_seed(0)
        model = MNISTMLP()
    else:
        from torchvision import datasets, transforms  # not installed on this image
        test_loader = torch.utils.data.DataLoader(
            datasets.MNIST('../data', train=False, transform=transforms.Compose([
                transforms.ToTensor(), transforms.Normalize((0.1307,), (0.3081,))])),
            batch_size=args.test_batch_size, shuffle=True)
        model = MNISTMLP()
        model.load_state_dict(torch.load(args.checkpoint, map_location='cpu',
                                         weights_only=True))

    settings = zip(args.wb, args.wt, args.db, args.dt, args.gs)

    results = {'accs': [], 'tmacs': [], 'param_bits': []}
    for wb, wt, db, dt, gs in settings:
        qmodel = deepcopy(model)
        qmodel.to(device)
        tr_params = static_linear_layer_settings(qmodel, wb, gs, wt)
        qmodel = replace_linear_layers(qmodel, tr_params, db, dt)

        # Profile (calibration)
        acc = test(args, qmodel, device, test_loader, pct=0.05)
        set_tr_tracking(qmodel, False)

        # Get results
        acc = test(args, qmodel, device, test_loader)
        acc = 100.0 * acc
        tmacs, param_bits = get_model_ops(qmodel, (torch.randn(1, 1, 28, 28, device=device),))
        results['accs'].append(acc)
        results['tmacs'].append(tmacs)
        results['param_bits'].append(param_bits)
        print(wb, wt, db, dt, gs, acc, tmacs, param_bits)

    if args.out_file:
        with open(args.out_file, 'w') as fp:
            json.dump(results, fp)
    return results


if __name__ == '__main__':
    main()
