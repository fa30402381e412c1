"""Evaluation helpers -- the reference's util.py (util.py:1-133): ``validate``, ``accuracy``,
``AverageMeter``, ``ProgressMeter``, ``get_imagenet_validation``; plus a synthetic
ImageNet-shaped loader (no dataset is available offline) and the distributed accuracy
reduction that replaces nn.DataParallel's gather-to-GPU0."""
import os
import time

import torch
import torch.distributed as dist


def get_imagenet_validation(args):
    """ImageFolder loader of ``<val_dir>/imagenet/val`` (util.py:11-36).  Needs torchvision
    and the dataset; with ``args.synthetic`` returns ``SyntheticImageNet`` instead."""
    if getattr(args, 'synthetic', False):
        return SyntheticImageNet(num_samples=getattr(args, 'num_samples', 1024),
                                 batch_size=args.batch_size,
                                 image_size=224, seed=getattr(args, 'seed', 0))
    try:
        import PIL
        import torchvision.datasets as datasets
        import torchvision.transforms as transforms
    except ImportError as e:
        raise RuntimeError("ImageNet loading needs torchvision + PIL (not installed); "
                           "run with --synthetic") from e
    normalize = transforms.Normalize(mean=[0.485, 0.456, 0.406], std=[0.229, 0.224, 0.225])
    if 'efficientnet' in args.arch:
        val_transforms = transforms.Compose([
            transforms.Resize(224, interpolation=PIL.Image.BICUBIC),
            transforms.CenterCrop(224), transforms.ToTensor(), normalize])
    else:
        val_transforms = transforms.Compose([
            transforms.Resize(256), transforms.CenterCrop(224), transforms.ToTensor(),
            normalize])
    return torch.utils.data.DataLoader(
        datasets.ImageFolder(os.path.join(args.val_dir, 'imagenet', 'val'), val_transforms),
        batch_size=args.batch_size, shuffle=False, num_workers=args.workers, pin_memory=True)


class _Targets(object):
    def __init__(self, n):
        self.targets = list(range(n))

    def __len__(self):
        return len(self.targets)


class SyntheticImageNet(object):
    """Deterministic N(0,1) 3x224x224 images with random labels in [0, 1000).

    Iterates like a DataLoader (``len``, ``.dataset.targets``).  With ``rank``/``world_size``
    it yields only batches rank, rank + world_size, ... (the static batch stride of the
    multi-GPU evaluation)."""

    def __init__(self, num_samples=1024, batch_size=256, image_size=224, seed=0, rank=0,
                 world_size=1, device='cpu'):
        self.num_samples = num_samples
        self.batch_size = batch_size
        self.image_size = image_size
        self.seed = seed
        self.rank = rank
        self.world_size = world_size
        self.device = device
        self.dataset = _Targets(num_samples)

    def __len__(self):
        return (self.num_samples + self.batch_size - 1) // self.batch_size

    def batch(self, i):
        n = min(self.batch_size, self.num_samples - i * self.batch_size)
        g = torch.Generator(device='cpu').manual_seed(self.seed * 1000003 + i)
        images = torch.randn(n, 3, self.image_size, self.image_size, generator=g)
        target = torch.randint(0, 1000, (n,), generator=g)
        return images.to(self.device), target.to(self.device)

    def __iter__(self):
        for i in range(self.rank, len(self), self.world_size):
            yield self.batch(i)


def validate(val_loader, model, criterion, args, verbose=True, pct=1.0):
    """Top-1 evaluation loop (util.py:39-80).  Under torch.distributed the loss and
    correct-count sums are all-reduced once at the end, so every rank returns the global
    figures (the reference reads GPU0's DataParallel gather)."""
    batch_time = AverageMeter('Time', ':6.3f')
    losses = AverageMeter('Loss', ':.4e')
    top1 = AverageMeter('Acc@1', ':6.2f')
    progress = ProgressMeter(len(val_loader), [batch_time, losses, top1], prefix='Test: ')

    model.eval()
    eval_samples = round(pct * len(val_loader.dataset.targets))
    curr_samples = 0
    world = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1

    with torch.no_grad():
        end = time.time()
        for i, (images, target) in enumerate(val_loader):
            if args.gpu is not None:
                images = images.cuda(args.gpu, non_blocking=True)
            curr_samples += len(target) * world
            if args.gpu is not None:
                target = target.cuda(args.gpu, non_blocking=True)

            output = model(images)
            loss = criterion(output, target)

            acc1 = accuracy(output, target, topk=1)
            losses.update(loss.item(), images.size(0))
            top1.update(acc1, images.size(0))

            batch_time.update(time.time() - end)
            end = time.time()

            if i % args.print_freq == 0 and verbose:
                progress.display(i)

            if curr_samples >= eval_samples:
                break

    if world > 1:
        dev = torch.device('cuda', args.gpu) if args.gpu is not None else torch.device('cpu')
        t = torch.tensor([losses.sum, top1.sum, float(top1.count)], dtype=torch.float64,
                         device=dev)
        dist.all_reduce(t)
        losses.avg = t[0].item() / max(t[2].item(), 1.0)
        top1.avg = t[1].item() / max(t[2].item(), 1.0)

    if verbose:
        print(' * Acc@1 {top1.avg:.3f} '.format(top1=top1))

    return losses.avg, top1.avg


class AverageMeter(object):
    """Computes and stores the average and current value"""

    def __init__(self, name, fmt=':f'):
        self.name = name
        self.fmt = fmt
        self.reset()

    def reset(self):
        self.val = 0
        self.avg = 0
        self.sum = 0
        self.count = 0

    def update(self, val, n=1):
        self.val = val
        self.sum += val * n
        self.count += n
        self.avg = self.sum / self.count

    def __str__(self):
        fmtstr = '{name} {val' + self.fmt + '} ({avg' + self.fmt + '})'
        return fmtstr.format(**self.__dict__)


class ProgressMeter(object):
    def __init__(self, num_batches, meters, prefix=""):
        self.batch_fmtstr = self._get_batch_fmtstr(num_batches)
        self.meters = meters
        self.prefix = prefix

    def display(self, batch):
        entries = [self.prefix + self.batch_fmtstr.format(batch)]
        entries += [str(meter) for meter in self.meters]
        print('\t'.join(entries))

    def _get_batch_fmtstr(self, num_batches):
        num_digits = len(str(num_batches // 1))
        fmt = '{:' + str(num_digits) + 'd}'
        return '[' + fmt + '/' + fmt.format(num_batches) + ']'


def accuracy(output, target, topk=1):
    '''Computes the accuracy over the k top predictions'''
    with torch.no_grad():
        batch_size = target.size(0)

        _, pred = output.topk(topk, 1, True, True)
        pred = pred.t()
        correct = pred.eq(target.view(1, -1).expand_as(pred))

        correct_k = correct[:topk].reshape(-1).float().sum(0, keepdim=True)
        return correct_k.mul_(100.0 / batch_size).item()


def allreduce_histograms(model):
    """Sum every TR layer's calibration histogram over all ranks (one collective for the
    whole model), so each rank's mse_profile sees the global activation distribution.
    The reference's DataParallel keeps only GPU0's replica updates (evaluate_cnn.py:33)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return
    import tr_layer
    quants = [m for m in model.modules() if isinstance(m, tr_layer.LinearQuantize)]
    if not quants:
        return
    flat = torch.stack([q.hist_bins for q in quants])
    dist.all_reduce(flat)
    for q, h in zip(quants, flat):
        q.hist_bins.copy_(h)
