"""The data-parallel evaluation path with real HIP kernels in every rank (BASELINE configs[4],
SURVEY 8(e)): evaluate_group_size.py --synthetic at world 1 and world 2, the two ranks sharing
the one MI355X of a test box (gloo collectives, TQ_DIST_BACKEND=gloo -- RCCL takes one rank per
GPU; the one-rank-per-GPU RCCL runs are the driver's 8-GPU bench).  Rank-strided batches,
calibration histograms all-reduced over the ranks and integer accuracy counters make every
(loss, top-1) pass and the results equal at both world sizes -- top-1, term-pair MACs and
average terms exactly; losses to fp32 rounding (each process picks its own MIOpen solver for
the fp32 stem conv, so per-batch losses may differ in the last bits across processes; the CPU
test, tests/test_dist.py, checks bit equality under gloo on the host)."""
import os
import socket

import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, out_dir, out):
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "term-quantization_amd"))
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port),
                       "RANK": str(rank), "LOCAL_RANK": "0", "WORLD_SIZE": str(world),
                       "TQ_DIST_BACKEND": "gloo"})
    import evaluate_cnn
    import evaluate_group_size
    evaluate_group_size.GROUP_SIZES = [1, 8, 32]
    evaluate_group_size.AVG_TERM_SETTINGS = [1.0, 3.0]
    seen = []
    validate = evaluate_cnn.util.validate

    def recording(*a, **k):
        r = validate(*a, **k)
        seen.append(r)
        return r
    evaluate_cnn.util.validate = recording
    res = evaluate_group_size.main(["--synthetic", "-a", "resnet18", "--gpu", "0",
                                    "--num-samples", "16", "-b", "4", "--image-size", "96",
                                    "--out-dir", out_dir])
    import torch
    out[rank] = (res, seen, torch.cuda.current_device())


def test_evaluate_group_size_two_ranks_on_the_gpu_equal_one(tmp_path):
    mgr = mp.Manager()
    runs = {}
    for world in (1, 2):
        out = mgr.dict()
        mp.spawn(_worker, args=(world, _free_port(), str(tmp_path / ("w%d" % world)), out),
                 nprocs=world, join=True)
        runs[world] = dict(out)
    r1, seen1, d1 = runs[1][0]
    r2, seen2, d2 = runs[2][0]
    assert d1 == d2 == 0 and runs[2][1][2] == 0  # every rank ran its kernels on cuda:0
    assert len(seen1) == 12 and len(seen2) == 12

    def close(a, b):
        if isinstance(a, dict):
            return a.keys() == b.keys() and all(close(a[k], b[k]) for k in a)
        if isinstance(a, (list, tuple)):
            return len(a) == len(b) and all(close(x, y) for x, y in zip(a, b))
        if isinstance(a, float):
            return abs(a - b) <= 1e-5 * max(1.0, abs(a))
        return a == b
    assert close(seen1, seen2) and [t for _, t in seen1] == [t for _, t in seen2]
    assert close(r1, r2)
    for g in r1:  # the integer-derived figures exactly
        assert r1[g]["tmacs"] == r2[g]["tmacs"] and r1[g]["avg_terms"] == r2[g]["avg_terms"]
    assert runs[2][1][0] == r2 and runs[2][1][1] == seen2  # both ranks hold the global figures
