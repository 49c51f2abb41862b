"""Skinny linear (mmpde_linear_skinny_ws, dense.hip): the res_cut / DMM-branch
GEMMs with K split over the chip and the partial tiles added in z order inside
the launch.

Bar: exact-fp32 products, so max|err| vs float64 <= 1e-6 x (1 + |ref|max)
times sqrt(k)/sqrt(512) slack; repeated calls bit-identical; one workspace
reused across shapes (the cylinder res_cut chain 2521-2048-512-2048-2521, then
shapes whose partial tiles cover other shapes' ticket words) stays exact and
leaves its ticket words at zero.
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

SHAPES = [(16, 2521, 2048), (16, 2048, 2521), (3, 2048, 2521), (3, 2521, 2048), (2, 512, 2048),
          (32, 2521, 512), (2, 4096, 64), (1, 100, 7), (64, 1024, 1000)]


def _ref(x, w, b, act):
    r = x.double() @ w.double().t() + b.double()
    return torch.tanh(r) if act == 1 else r


def _bound(ref, k):
    return 1e-6 * (1 + ref.abs().max().item()) * max(1.0, math.sqrt(k / 512))


@pytest.mark.parametrize("m,k,n", SHAPES)
def test_linear_skinny_vs_fp64(dev, m, k, n):
    from mmpde_amd import ops

    g = torch.Generator().manual_seed(m * 7 + k + n)
    x = torch.randn(m, k, generator=g).to(dev)
    w = (torch.randn(n, k, generator=g) * 0.02).to(dev)
    b = torch.randn(n, generator=g).to(dev)
    for act in (0, 1):
        ref = _ref(x, w, b, act)
        outs = [ops.linear_skinny(x, w, b, act) for _ in range(3)]
        err = (outs[0].double() - ref.to(dev)).abs().max().item()
        assert err <= _bound(ref, k), (m, k, n, act, err)
        assert all(torch.equal(outs[0], o) for o in outs[1:]), "run-to-run"


def test_linear_skinny_workspace_reuse(dev):
    from mmpde_amd import _lib as L, ops

    g = torch.Generator().manual_seed(3)
    widths = [2521, 2048, 512, 2048, 2521]
    layers = [((torch.randn(b_, a_, generator=g) * 0.02).to(dev), torch.randn(b_, generator=g).to(dev))
              for a_, b_ in zip(widths, widths[1:])]
    for m in (2, 3, 16):
        x = torch.randn(m, 2521, generator=g).to(dev)
        for _ in range(2):
            h, r = x, x.double()
            for i, (w, b) in enumerate(layers):
                act = 1 if i < 3 else 0
                h = ops.linear_skinny(h, w, b, act)
                r = _ref(r, w, b, act)
                err = (h.double() - r).abs().max().item()
                assert err <= _bound(r, w.shape[1]), (m, i, err)
    torch.cuda.synchronize()
    assert L.lib().mmpde_linear_skinny_workspace_bytes(16, 2521, 2048) > 4096 * 4
    for ws in ops._SKINNY_WS.values():
        assert int(ws[:4096].view(torch.int32).abs().sum()) == 0, "ticket words left non-zero"


CHAINS = [
    # res_cut (interpolate.py:66-74): 2521-2048-512-2048-2521, tanh x3
    ([2521, 2048, 512, 2048, 2521], [1, 1, 1, 0]),
    # DMM output_mlp + P (mesh/dmm_model.py:175-181): N-512-256-L, then L -> hidden
    ([2521, 512, 256, 64, 512], [1, 1, 0, 0]),
    ([2304, 1024, 64, 512], [1, 0, 0]),          # array branch fc2, fc3 + P
    ([100, 7], [2]),                             # one layer, ragged widths
    ([5, 33, 17, 1], [1, 2, 0]),
]


def _chain_layers(dims, acts, g, dev):
    return [((torch.randn(b_, a_, generator=g) * (1.0 / math.sqrt(a_))).to(dev),
             torch.randn(b_, generator=g).to(dev) * 0.1, act)
            for a_, b_, act in zip(dims, dims[1:], acts)]


@pytest.mark.parametrize("ci", range(len(CHAINS)))
@pytest.mark.parametrize("m", [1, 16, 33, 64])
def test_linear_chain_vs_fp64(dev, ci, m):
    """mmpde_linear_chain_ws: every layer of the chain in one launch (grid
    barrier between layers) against float64 layer by layer; run to run
    bit-identical; the counters left at zero (the workspace is reused)."""
    from mmpde_amd import ops

    dims, acts = CHAINS[ci]
    g = torch.Generator().manual_seed(100 * ci + m)
    layers = _chain_layers(dims, acts, g, dev)
    x = torch.randn(m, dims[0], generator=g).to(dev)
    r = x.double()
    for w, b, act in layers:
        r = r @ w.double().t() + b.double()
        r = torch.tanh(r) if act == 1 else (torch.relu(r) if act == 2 else r)
    outs = [ops.linear_chain(x, layers) for _ in range(3)]
    # error grows through the chain: the fp32 bound of each layer's K, summed
    bound = sum(_bound(r, k) for k in dims[:-1]) * 4
    err = (outs[0].double() - r).abs().max().item()
    assert err <= bound, (dims, m, err, bound)
    assert all(torch.equal(outs[0], o) for o in outs[1:]), "run-to-run"
    torch.cuda.synchronize()
    for ws in ops._CHAIN_WS.values():
        assert int(ws[:4096].view(torch.int32).abs().sum()) == 0, "control words left non-zero"


def test_linear_chain_rows_independent(dev):
    """A row's result does not depend on the rows launched beside it (the K
    split depends on (n, k) only): the sharded evaluation's bitwise bar."""
    from mmpde_amd import ops

    dims, acts = CHAINS[0]
    g = torch.Generator().manual_seed(7)
    layers = _chain_layers(dims, acts, g, dev)
    x = torch.randn(16, dims[0], generator=g).to(dev)
    full = ops.linear_chain(x, layers)
    assert torch.equal(full[:8], ops.linear_chain(x[:8].contiguous(), layers))
    assert torch.equal(full[8:], ops.linear_chain(x[8:].contiguous(), layers))
    assert torch.equal(full[5:6], ops.linear_chain(x[5:6].contiguous(), layers))


def test_res_cut_chain_matches_skinny_layers(dev):
    """ItpNet.res_cut (cylinder MLP) through the chain agrees with the four
    separate skinny launches to fp32 rounding (same per-item arithmetic, the
    K splits may differ)."""
    from mmpde_amd import ops

    dims, acts = CHAINS[0]
    g = torch.Generator().manual_seed(11)
    layers = _chain_layers(dims, acts, g, dev)
    x = torch.randn(16, dims[0], generator=g).to(dev)
    h = x
    for w, b, act in layers:
        h = ops.linear_skinny(h, w, b, act)
    c = ops.linear_chain(x, layers)
    assert (c - h).abs().max().item() <= 1e-5 * (1 + h.abs().max().item())


@pytest.mark.parametrize("m", [3, 16])
def test_linear_chain_reused_workspace_new_inputs(dev, m):
    """One workspace, many launches with NEW inputs each time (the rollout's
    pattern): every launch against float64, with another chain interleaved
    on the same stream."""
    from mmpde_amd import ops

    g = torch.Generator().manual_seed(23 + m)
    chains = [_chain_layers(*CHAINS[i], g, dev) for i in (0, 1)]
    for it in range(6):
        for ci, layers in enumerate(chains):
            dims = CHAINS[(0, 1)[ci]][0]
            x = torch.randn(m, dims[0], generator=g).to(dev)
            r = x.double()
            for w, b, act in layers:
                r = r @ w.double().t() + b.double()
                r = torch.tanh(r) if act == 1 else r
            y = ops.linear_chain(x, layers)
            err = (y.double() - r).abs().max().item()
            bound = sum(_bound(r, k) for k in dims[:-1]) * 4
            assert err <= bound, (it, ci, m, err, bound)


def test_linear_chain_under_uneven_load(dev):
    """The in-launch hand-offs under uneven load (guide: test every hand-off
    with other work on the chip): chains on one stream, large GEMMs on another,
    new inputs every launch, each checked against float64; the barrier's
    timeout word stays clear."""
    from mmpde_amd import ops

    g = torch.Generator().manual_seed(5)
    dims, acts = CHAINS[0]
    layers = _chain_layers(dims, acts, g, dev)
    s_chain, s_load = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    big = torch.randn(4096, 4096, device=dev)
    outs, refs, xs = [], [], []   # inputs kept alive: read on s_chain, allocated on the default stream
    for it in range(8):
        x = torch.randn(3, dims[0], generator=g).to(dev)
        xs.append(x)
        r = x.double()
        for w, b, act in layers:
            r = r @ w.double().t() + b.double()
            r = torch.tanh(r) if act == 1 else r
        refs.append(r)
        torch.cuda.synchronize(dev)
        with torch.cuda.stream(s_load):
            for _ in range(3):
                big = torch.tanh(big @ big * 1e-3)
        with torch.cuda.stream(s_chain):
            outs.append(ops.linear_chain(x, layers))
    torch.cuda.synchronize(dev)
    bound = sum(_bound(refs[0], k) for k in dims[:-1]) * 4
    for it, (y, r) in enumerate(zip(outs, refs)):
        err = (y.double() - r).abs().max().item()
        assert err <= bound, (it, err, bound)
    for ws in ops._CHAIN_WS.values():
        assert int(ws[:4096].view(torch.int32).abs().sum()) == 0, "control / timeout words left non-zero"


def test_linear_chains_concurrent_streams(dev):
    """Two chains in flight at once on two streams, grids larger than half the
    chip each: a workgroup only ever waits for items claimed before its own,
    so concurrent chains cannot starve each other (the failure mode of a grid
    barrier); every result against float64."""
    from mmpde_amd import ops

    g = torch.Generator().manual_seed(9)
    specs = [CHAINS[0], CHAINS[1]]
    chains = [_chain_layers(d, a, g, dev) for d, a in specs]
    streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    xs = [(ci, torch.randn(16, specs[ci][0][0], generator=g).to(dev)) for it in range(6) for ci in (0, 1)]
    for ci in (0, 1):   # workspaces allocated (zeroed) before the concurrent launches
        with torch.cuda.stream(streams[ci]):
            ops.linear_chain(xs[ci][1], chains[ci])
    torch.cuda.synchronize(dev)
    outs = []
    for ci, x in xs:   # launched back to back, no synchronisation in between
        with torch.cuda.stream(streams[ci]):
            outs.append(ops.linear_chain(x, chains[ci]))
    torch.cuda.synchronize(dev)
    for (ci, x), y in zip(xs, outs):
        r = x.double()
        for w, b, act in chains[ci]:
            r = r @ w.double().t() + b.double()
            r = torch.tanh(r) if act == 1 else r
        bound = sum(_bound(r, k) for k in specs[ci][0][:-1]) * 4
        assert (y.double() - r).abs().max().item() <= bound
    for ws in ops._CHAIN_WS.values():
        assert int(ws[:4096].view(torch.int32).abs().sum()) == 0, "control / timeout words left non-zero"
