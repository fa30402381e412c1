"""Evaluation helpers -- the reference's util.py roles (util.py:1-133): ``validate``,
``accuracy``, ``get_imagenet_validation`` (its AverageMeter/ProgressMeter printing is folded
into validate's progress line); plus a synthetic
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
    """Top-1 evaluation loop over (pct of) the loader (util.py:39-80): returns (mean loss,
    top-1 %) weighted by batch size.  Under torch.distributed the loss / correct / sample
    sums are all-reduced once at the end, so every rank returns the global figures (the
    reference reads GPU0's DataParallel gather)."""
    model.eval()
    eval_samples = round(pct * len(val_loader.dataset.targets))
    world = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
    seen = 0
    totals = [0.0, 0.0, 0.0]  # sum of loss * n, sum of top-1 % * n, n (this rank)
    tick = time.time()
    with torch.no_grad():
        for i, (images, target) in enumerate(val_loader):
            if args.gpu is not None:
                images = images.cuda(args.gpu, non_blocking=True)
                target = target.cuda(args.gpu, non_blocking=True)
            seen += len(target) * world
            output = model(images)
            n = images.size(0)
            loss, acc1 = criterion(output, target).item(), accuracy(output, target, topk=1)
            totals[0] += loss * n
            totals[1] += acc1 * n
            totals[2] += n
            if verbose and i % args.print_freq == 0:  # batch value (running mean)
                now = time.time()
                print("Test: [%d/%d]\tTime %.3f\tLoss %.4e (%.4e)\tAcc@1 %.2f (%.2f)" % (
                    i, len(val_loader), now - tick, loss, totals[0] / totals[2], acc1,
                    totals[1] / totals[2]))
                tick = now
            if seen >= eval_samples:
                break
    if world > 1:
        dev = torch.device('cuda', args.gpu) if args.gpu is not None else torch.device('cpu')
        t = torch.tensor(totals, dtype=torch.float64, device=dev)
        dist.all_reduce(t)
        totals = t.tolist()
    loss = totals[0] / max(totals[2], 1.0)
    top1 = totals[1] / max(totals[2], 1.0)
    if verbose:
        print(' * Acc@1 %.3f ' % top1)
    return loss, top1


def accuracy(output, target, topk=1):
    """Percentage of rows whose target is among the ``topk`` highest outputs (the
    reference's util.accuracy for one k, util.py:123-133)."""
    with torch.no_grad():
        hits = (output.topk(topk, dim=1).indices == target.view(-1, 1)).any(dim=1)
        return 100.0 * hits.float().mean().item()


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
