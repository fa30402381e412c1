"""CPU restatement of the stream-K work split and fixup bookkeeping of
csrc/tr_conv.hip (conv2d_tp_streamk_kernel / conv2d_tp_streamk_fixup): every (tile,
K-step) unit is summed exactly once and every tile gets exactly one epilogue."""
import pytest


def plan(tiles, nsteps, G):
    U = tiles * nsteps
    bound = lambda b: b * U // G  # noqa: E731
    units = {}
    epilogues = {}
    slabs = {}
    for b in range(G):
        u0, u1 = bound(b), bound(b + 1)
        u = u0
        while u < u1:
            t = u // nsteps
            k0 = u - t * nsteps
            k1 = min(nsteps, k0 + (u1 - u))
            for k in range(k0, k1):
                units[(t, k)] = units.get((t, k), 0) + 1
            if k0 == 0 and k1 == nsteps:
                epilogues[t] = epilogues.get(t, 0) + 1
            else:
                slot = 0 if u == u0 else 1
                assert (b, slot) not in slabs
                slabs[(b, slot)] = (t, set(range(k0, k1)))
            u += k1 - k0
    # fixup: one block per inner boundary
    for b in range(1, G):
        ub = bound(b)
        if ub % nsteps == 0 or ub >= U:
            continue
        t = ub // nsteps
        if bound(b - 1) > t * nsteps:
            continue
        covered = set()
        bb = b - 1
        while bb < G and bound(bb) < (t + 1) * nsteps:
            if bound(bb + 1) > t * nsteps:
                slot = 0 if bound(bb) // nsteps == t else 1
                st, ks = slabs[(bb, slot)]
                assert st == t and not (covered & ks)
                covered |= ks
            bb += 1
        assert covered == set(range(nsteps)), (t, covered)
        epilogues[t] = epilogues.get(t, 0) + 1
    assert all(units.get((t, k)) == 1 for t in range(tiles) for k in range(nsteps))
    assert all(epilogues.get(t) == 1 for t in range(tiles)), epilogues


@pytest.mark.parametrize("tiles,nsteps,G", [(1568, 36, 768), (392, 144, 768), (3136, 18, 768),
                                             (784, 72, 768), (7, 5, 768), (100, 3, 7),
                                             (5, 144, 3), (10, 1, 4), (1, 64, 9)])
def test_streamk_plan_covers_every_unit_once(tiles, nsteps, G):
    plan(tiles, nsteps, min(G, tiles * nsteps))
