"""Evaluation helpers -- the reference's util.py roles (util.py:1-133): ``validate``,
``accuracy``, ``get_imagenet_validation`` (its AverageMeter/ProgressMeter printing is folded
into validate's progress line); plus a synthetic
ImageNet-shaped loader (no dataset is available offline) and the distributed accuracy
reduction that replaces nn.DataParallel's gather-to-GPU0."""
import os
import time

import torch
import torch.distributed as dist


class StridedBatchSampler(object):
    """Batches of consecutive sample indices [i*bs, (i+1)*bs) for the global batch indices
    i = rank, rank + world, ... -- the static batch stride of the multi-GPU evaluation
     applied to a map-style dataset: no padding and no duplicated samples,
    so the all-reduced counters cover every sample exactly once (unlike a padded
    DistributedSampler), and the union over ranks is the unsharded loader's batches."""

    def __init__(self, num_samples, batch_size, rank=0, world_size=1):
        self.num_samples, self.batch_size = int(num_samples), int(batch_size)
        self.rank, self.world_size = int(rank), int(world_size)

    def __len__(self):
        nb = (self.num_samples + self.batch_size - 1) // self.batch_size
        return len(range(self.rank, nb, self.world_size))

    def __iter__(self):
        nb = (self.num_samples + self.batch_size - 1) // self.batch_size
        for i in range(self.rank, nb, self.world_size):
            yield list(range(i * self.batch_size,
                             min((i + 1) * self.batch_size, self.num_samples)))


class ShardedLoader(object):
    """A DataLoader over one rank's strided batches (StridedBatchSampler) that keeps the
    attributes validate() relies on: ``dataset`` (``.targets``), ``batch_size``, ``rank``,
    ``world_size`` and ``len`` = the GLOBAL batch count, as SyntheticImageNet does."""

    def __init__(self, dataset, batch_size, rank=0, world_size=1, **loader_kwargs):
        import torch.utils.data
        self.dataset, self.batch_size = dataset, batch_size
        self.rank, self.world_size = rank, world_size
        self.sampler = StridedBatchSampler(len(dataset), batch_size, rank, world_size)
        self.loader = torch.utils.data.DataLoader(dataset, batch_sampler=self.sampler,
                                                  **loader_kwargs)

    def __len__(self):
        return (len(self.dataset) + self.batch_size - 1) // self.batch_size

    def __iter__(self):
        return iter(self.loader)


def get_imagenet_validation(args, rank=0, world_size=1):
    """ImageFolder loader of ``<val_dir>/imagenet/val`` (util.py:11-36).  Needs torchvision
    and the dataset; with ``args.synthetic`` returns ``SyntheticImageNet`` instead.  Either
    way, ``rank``/``world_size`` shard it by the static batch stride (StridedBatchSampler)."""
    if getattr(args, 'synthetic', False):
        return SyntheticImageNet(num_samples=getattr(args, 'num_samples', 1024),
                                 batch_size=args.batch_size,
                                 image_size=getattr(args, 'image_size', 224),
                                 seed=getattr(args, 'seed', 0), rank=rank,
                                 world_size=world_size)
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
    return ShardedLoader(
        datasets.ImageFolder(os.path.join(args.val_dir, 'imagenet', 'val'), val_transforms),
        args.batch_size, rank, world_size, num_workers=args.workers, pin_memory=True)


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
    top-1 %) over the samples seen.  The reference runs batches until the samples seen reach
    pct of the dataset; here that rule is applied to GLOBAL batch indices, so a loader sharded
    over ranks (SyntheticImageNet / ShardedLoader: rank r holds batches r, r + world, ...)
    covers exactly the batches the unsharded loader would.  Under torch.distributed the loss
    sum and the integer correct / sample counts are all-reduced once at the end, so every rank
    returns the global figures (the reference reads GPU0's DataParallel gather)."""
    model.eval()
    eval_samples = round(pct * len(val_loader.dataset.targets))
    world = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
    shard_rank = getattr(val_loader, 'rank', 0)
    shard_world = getattr(val_loader, 'world_size', 1)
    if shard_world != world:
        raise ValueError("validate: the loader is sharded over %d ranks but the process group "
                         "has %d" % (shard_world, world))
    bs = val_loader.batch_size
    loss_sum, correct, count = 0.0, 0, 0  # this rank
    tick = time.time()
    with torch.no_grad():
        for i, (images, target) in enumerate(val_loader):
            gi = shard_rank + i * shard_world  # global batch index
            if gi > 0 and gi * bs >= eval_samples:
                break  # the unsharded loop stopped after global batch gi - 1
            if args.gpu is not None:
                images = images.cuda(args.gpu, non_blocking=True)
                target = target.cuda(args.gpu, non_blocking=True)
            output = model(images)
            n = images.size(0)
            loss = criterion(output, target).item()
            hits = correct_count(output, target, topk=1)
            loss_sum += loss * n
            correct += hits
            count += n
            if verbose and i % args.print_freq == 0:  # batch value (running mean)
                now = time.time()
                print("Test: [%d/%d]\tTime %.3f\tLoss %.4e (%.4e)\tAcc@1 %.2f (%.2f)" % (
                    gi, len(val_loader), now - tick, loss, loss_sum / count, 100.0 * hits / n,
                    100.0 * correct / count))
                tick = now
    if world > 1:
        dev = torch.device('cuda', args.gpu) if args.gpu is not None else torch.device('cpu')
        t = torch.tensor([loss_sum], dtype=torch.float64, device=dev)
        c = torch.tensor([correct, count], dtype=torch.int64, device=dev)
        all_reduce_sum(t)
        all_reduce_sum(c)
        loss_sum = float(t.item())
        correct, count = (int(v) for v in c.tolist())
    loss = loss_sum / max(count, 1)
    top1 = 100.0 * correct / max(count, 1)
    if verbose:
        print(' * Acc@1 %.3f ' % top1)
    return loss, top1


def correct_count(output, target, topk=1):
    """Rows whose target is among the ``topk`` highest outputs (an exact integer, so
    per-rank counts all-reduce to exactly the single-process count)."""
    with torch.no_grad():
        return int((output.topk(topk, dim=1).indices == target.view(-1, 1)).any(dim=1).sum())


def accuracy(output, target, topk=1):
    """Percentage of rows whose target is among the ``topk`` highest outputs (the
    reference's util.accuracy for one k, util.py:123-133)."""
    with torch.no_grad():
        hits = (output.topk(topk, dim=1).indices == target.view(-1, 1)).any(dim=1)
        return 100.0 * hits.float().mean().item()


def all_reduce_sum(t):
    """In-place sum over the ranks: RCCL on device tensors; under gloo (CPU ranks, or ranks
    sharing one GPU: evaluate_cnn TQ_DIST_BACKEND=gloo) a device tensor goes through a host
    copy."""
    if t.is_cuda and dist.get_backend() == "gloo":
        h = t.cpu()
        dist.all_reduce(h)
        t.copy_(h)
    else:
        dist.all_reduce(t)


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
    all_reduce_sum(flat)
    for q, h in zip(quants, flat):
        q.hist_bins.copy_(h)
