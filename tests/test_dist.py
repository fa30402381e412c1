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


def _grid_worker(rank, world, port, out_dir, out):
    """One torchrun-style rank of evaluate_group_size.py on the CPU (--gpu -1: gloo)."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "term-quantization_amd"))
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port),
                       "RANK": str(rank), "LOCAL_RANK": str(rank), "WORLD_SIZE": str(world)})
    torch.set_num_threads(max(1, 8 // world))
    import evaluate_cnn
    import evaluate_group_size
    # a corner subset of the 25-point grid keeps the CPU suite short (the whole grid runs at
    # world 1 under -m gpu, tests/test_gpu_grid.py); the sharding is what is checked here
    evaluate_group_size.GROUP_SIZES = [1, 32]
    evaluate_group_size.AVG_TERM_SETTINGS = [1.0, 3.0]
    seen = []
    validate = evaluate_cnn.util.validate

    def recording(*a, **k):  # (loss, top1) of every calibration / evaluation pass
        r = validate(*a, **k)
        seen.append(r)
        return r
    evaluate_cnn.util.validate = recording
    res = evaluate_group_size.main(["--synthetic", "-a", "resnet18", "--gpu", "-1",
                                    "--num-samples", "6", "-b", "2", "--image-size", "64",
                                    "--out-dir", out_dir])
    out[rank] = (res, seen)


def test_evaluate_group_size_world2_equals_world1(tmp_path):
    """BASELINE configs[4] through the code torchrun launches: evaluate_group_size.py --synthetic
    on the CPU (gloo) at world 1 and world 2.  Rank-strided batches, histograms summed over
    ranks and integer counters make the results JSON -- and every (loss, top-1) pass of the
    grid-corner settings -- identical at both world sizes; the written file equals the returned dict."""
    import json
    mgr = mp.Manager()
    runs = {}
    for world in (1, 2):
        out = mgr.dict()
        d = str(tmp_path / ("w%d" % world))
        mp.spawn(_grid_worker, args=(world, _free_port(), d, out), nprocs=world, join=True)
        runs[world] = dict(out)
        written = json.load(open(os.path.join(d, "resnet18-group-size-results.json")))
        assert written == runs[world][0][0]
    r1, seen1 = runs[1][0]
    r2, seen2 = runs[2][0]
    assert r1 == r2 and seen1 == seen2 and len(seen1) == 8
    assert runs[2][1] == runs[2][0]  # both ranks return the global figures
    pub = json.load(open(os.path.join(HERE, "golden", "published_results.json")))[
        "resnet18-group-size-results.json"]
    for g in ("1", "32"):  # the published term-pair MAC counts per setting (avg 1.0 and 3.0)
        assert r1[g]["tmacs"] == [pub[g]["tmacs"][i] for i in (0, 4)]
        assert r1[g]["avg_terms"] == [pub[g]["avg_terms"][i] for i in (0, 4)]


def test_sharded_loader_covers_a_map_style_dataset_once():
    """The ImageFolder path's sharding (util.ShardedLoader / StridedBatchSampler) on a
    map-style dataset: ranks hold the strided global batches, unpadded, and together they are
    exactly the unsharded loader's batches -- no duplicated samples in the counters."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "term-quantization_amd"))
    import util
    ds = torch.utils.data.TensorDataset(torch.arange(23).float(), torch.arange(23))
    ds.targets = list(range(23))
    full = [y.tolist() for _, y in torch.utils.data.DataLoader(ds, batch_size=4)]
    for world in (1, 2, 3, 8):
        shards = [util.ShardedLoader(ds, 4, r, world) for r in range(world)]
        got = {}
        for r, sh in enumerate(shards):
            assert len(sh) == len(full) and sh.batch_size == 4 and sh.world_size == world
            for j, (_, y) in enumerate(sh):
                got[r + j * world] = y.tolist()
        assert [got[i] for i in range(len(full))] == full
