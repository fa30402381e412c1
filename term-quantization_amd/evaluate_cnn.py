"""CNN uniform-quantization (UQ) / term-quantization (TQ) sweep -- the reference's
evaluate_cnn.py (evaluate_cnn.py:1-130) with the same command line and result JSON.

    python evaluate_cnn.py <val_dir> -a resnet18 -b 256 --gpu 0
    python evaluate_cnn.py --synthetic -a resnet18 -b 256            # no dataset offline
    torchrun --nproc-per-node 8 evaluate_cnn.py --synthetic -a resnet18

Multi-GPU: one process per GPU (torch.distributed, RCCL) instead of nn.DataParallel; every
rank evaluates its own share of the validation batches, the calibration histograms are
summed across ranks before the scale-factor search, and the accuracy counters are
all-reduced once per setting.
"""
import argparse
import json
import os
from copy import deepcopy

import torch
import torch.distributed as dist
import torch.nn as nn

import cnn_models
import profile_model
import tr_layer
import util


def compute_avg_terms(tr_params):
    alphas = []
    for weight_bits, group_size, weight_terms in tr_params[1:]:
        alphas.append(weight_terms / group_size)

    return sum(alphas) / len(alphas)


def _rank():
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0


def eval_model(args, model, weight_bits, group_size, weight_terms, data_bits, data_terms):
    """Convert, count term-pair MACs, calibrate, evaluate (evaluate_cnn.py:20-42).  The
    calibration pass sees pct=0.05 of the set, i.e. the same global batches at any world
    size; the histograms are summed over ranks before the scale-factor search."""
    tr_params = cnn_models.static_conv_layer_settings(model, weight_bits,
                                                      group_size, weight_terms)
    avg_terms = compute_avg_terms(tr_params)
    qmodel = cnn_models.convert_model(model, tr_params, data_bits, data_terms)
    if args.channels_last:
        qmodel = qmodel.to(memory_format=torch.channels_last)
    qmt = deepcopy(qmodel)
    x = torch.randn(1, 3, 224, 224, device=next(qmodel.parameters()).device)
    tmacs, params = profile_model.get_model_ops(qmt, (x,))
    del qmt

    # compute activation scale factors (histograms summed over ranks)
    _ = util.validate(val_loader, qmodel, criterion, args, verbose=args.verbose, pct=0.05)
    util.allreduce_histograms(qmodel)
    tr_layer.set_tr_tracking(qmodel, False)

    # evaluate model performance
    _, acc = util.validate(val_loader, qmodel, criterion, args, verbose=args.verbose)

    return acc, tmacs, avg_terms, params


def build_parser(description='PyTorch ImageNet Training'):
    parser = argparse.ArgumentParser(description=description)
    parser.add_argument('val_dir', nargs='?', default=None,
                        help='path to validation data folder')
    parser.add_argument('-a', '--arch', metavar='ARCH', default='alexnet',
                        choices=cnn_models.model_names(),
                        help='model architecture: ' +
                        ' | '.join(cnn_models.model_names()) +
                        ' (default: resnet18)')
    parser.add_argument('-j', '--workers', default=4, type=int, metavar='N',
                        help='number of data loading workers (default: 4)')
    parser.add_argument('-b', '--batch-size', default=256, type=int,
                        metavar='N', help='mini-batch size (default: 256)')
    parser.add_argument('-p', '--print-freq', default=10, type=int,
                        metavar='N', help='print frequency (default: 10)')
    parser.add_argument('--gpu', default=None, type=int,
                        help='GPU id to use (-1: run on the CPU, gloo between ranks).')
    parser.add_argument('-v', '--verbose', action='store_true', help='verbose flag')
    # additions: offline operation and output location
    parser.add_argument('--synthetic', action='store_true',
                        help='synthetic N(0,1) images + random-init weights (no dataset)')
    parser.add_argument('--num-samples', default=1024, type=int,
                        help='synthetic validation set size')
    parser.add_argument('--image-size', default=224, type=int,
                        help='synthetic image size (the term-pair MAC count is always taken '
                             'at 224x224, evaluate_cnn.py:28-29)')
    parser.add_argument('--seed', default=0, type=int)
    parser.add_argument('--out-dir', default='results')
    parser.add_argument('--channels-last', action='store_true',
                        help='run the network in channels_last (NHWC) memory format')
    return parser


def setup(args):
    """Device, process group, loader, criterion and the fp32 model.

    One process per device under torchrun: RCCL ("nccl") on GPUs, gloo on the CPU
    (``--gpu -1``, or no GPU present); TQ_DIST_BACKEND=gloo selects gloo on GPUs too (ranks
    sharing one device, as tests/test_gpu_dist.py runs them: RCCL takes one rank per GPU).  Every rank evaluates its own strided share of the
    batches -- the synthetic set and the ImageFolder alike (util.StridedBatchSampler) -- so
    the all-reduced counters cover each sample exactly once."""
    global val_loader, criterion
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    use_cpu = (args.gpu is not None and args.gpu < 0) or not torch.cuda.is_available()
    if use_cpu:
        args.gpu = None
        dev = torch.device('cpu')
    else:
        if world > 1:
            args.gpu = int(os.environ.get('LOCAL_RANK', '0'))
        if args.gpu is None:
            args.gpu = 0
        torch.cuda.set_device(args.gpu)
        dev = torch.device('cuda', args.gpu)
    if world > 1:
        if use_cpu:
            dist.init_process_group('gloo')
        elif os.environ.get('TQ_DIST_BACKEND', 'nccl') == 'gloo':
            dist.init_process_group('gloo')
        else:
            dist.init_process_group('nccl', device_id=dev)
    val_loader = util.get_imagenet_validation(args, rank=_rank(), world_size=world)
    criterion = nn.CrossEntropyLoss().to(dev)
    torch.manual_seed(args.seed)
    model = cnn_models.__dict__[args.arch](pretrained=not args.synthetic).to(dev)
    model.eval()
    return model


def finish():
    """Tear the process group down (torchrun ranks)."""
    if dist.is_available() and dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


def save(args, results, name):
    if _rank() == 0:
        os.makedirs(args.out_dir, exist_ok=True)
        with open(os.path.join(args.out_dir, name), 'w') as fp:
            json.dump(results, fp)


val_loader = None
criterion = None

if __name__ == '__main__':
    args = build_parser().parse_args()
    model = setup(args)

    results = {
        'quant': {'accs': [], 'tmacs': [], 'avg_terms': [], 'params': []},
        'tr-data2': {'accs': [], 'tmacs': [], 'avg_terms': [], 'params': []},
        'tr-data3': {'accs': [], 'tmacs': [], 'avg_terms': [], 'params': []},
        'tr-data4': {'accs': [], 'tmacs': [], 'avg_terms': [], 'params': []},
    }

    # Traditional Quantization Settings (evaluate_cnn.py:94-108)
    weight_bits = 9
    group_size = 1
    weight_terms = 9
    data_bits = 9
    data_terms = 9
    weight_bit_settings = [6, 7, 8, 9]
    for weight_bits in weight_bit_settings:
        res = eval_model(args, model, weight_bits, group_size, weight_terms,
                         data_bits, data_terms)
        acc, tmacs, avg_terms, params = res
        print(tmacs, acc)
        results['quant']['accs'].append(acc)
        results['quant']['tmacs'].append(tmacs)
        results['quant']['avg_terms'].append(avg_terms)
        results['quant']['params'].append(params)

    # Term Revealing Settings (evaluate_cnn.py:110-127)
    weight_bits = 9
    group_size = 8
    data_bits = 9
    data_term_settings = [2, 3, 4]
    weight_term_settings = [12, 16, 20, 24]
    for data_terms in data_term_settings:
        key = 'tr-data{}'.format(data_terms)
        for weight_terms in weight_term_settings:
            res = eval_model(args, model, weight_bits, group_size,
                             weight_terms, data_bits, data_terms)
            acc, tmacs, avg_terms, params = res
            print(tmacs, acc)
            results[key]['accs'].append(acc)
            results[key]['tmacs'].append(tmacs)
            results[key]['avg_terms'].append(avg_terms)
            results[key]['params'].append(params)

    save(args, results, '{}-results.json'.format(args.arch))
    finish()
