"""Multi-process (world_size 2, gloo, CPU) checks of the data-parallel evaluation path:
batch sharding, the calibration-histogram all-reduce and the accuracy-counter reduction that
replace nn.DataParallel (evaluate_cnn.py:33) -- the same code runs over RCCL on GPUs."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn as nn

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, out):
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "term-quantization_amd"))
    import tr_layer
    import util
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # 1) sharding: ranks see disjoint, strided batches covering the set
        loader = util.SyntheticImageNet(num_samples=40, batch_size=8, image_size=4, seed=3,
                                        rank=rank, world_size=world)
        seen = [y.tolist() for _, y in loader]
        # 2) histogram all-reduce over every LinearQuantize of a model
        model = nn.Sequential(tr_layer.LinearQuantize(9, 3), tr_layer.LinearQuantize(9, 3))
        torch.manual_seed(rank)
        for q in model:
            q(torch.randn(1000) * (rank + 1))
        local = torch.stack([q.hist_bins.clone() for q in model])
        util.allreduce_histograms(model)
        merged = torch.stack([q.hist_bins for q in model])
        # 3) validate(): global accuracy from per-rank counters
        torch.manual_seed(0)
        net = nn.Sequential(nn.Flatten(), nn.Linear(3 * 4 * 4, 1000))

        class A:
            gpu = None
            print_freq = 1000
        _, acc = util.validate(loader, net, nn.CrossEntropyLoss(), A(), verbose=False)
        out[rank] = (seen, local, merged, acc)
    finally:
        dist.destroy_process_group()


def test_gloo_world2_sharding_histograms_accuracy():
    world = 2
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, port, out), nprocs=world, join=True)
    seen0, local0, merged0, acc0 = out[0]
    seen1, local1, merged1, acc1 = out[1]
    # disjoint shards that together cover all 5 batches
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "term-quantization_amd"))
    import util
    full = util.SyntheticImageNet(num_samples=40, batch_size=8, image_size=4, seed=3)
    all_batches = [full.batch(i)[1].tolist() for i in range(len(full))]
    assert seen0 == all_batches[0::2] and seen1 == all_batches[1::2]
    # every rank holds the sum of both ranks' histograms
    assert torch.equal(merged0, local0 + local1) and torch.equal(merged1, merged0)
    # both ranks report the same global accuracy, equal to the single-process value
    assert acc0 == pytest.approx(acc1)
    torch.manual_seed(0)
    net = nn.Sequential(nn.Flatten(), nn.Linear(3 * 4 * 4, 1000))
    correct = total = 0
    for i in range(len(full)):
        x, y = full.batch(i)
        correct += (net(x).argmax(1) == y).sum().item()
        total += y.numel()
    assert acc0 == pytest.approx(100.0 * correct / total)
