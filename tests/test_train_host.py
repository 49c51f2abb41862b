"""Host-side pieces of the training path (no GPU): the reverse adjacency the
edge-stage backward sums source gradients over, and the oracle's train-mode
forward (BatchNorm on batch statistics, running buffers updated in place)."""
import torch

from mmpde_amd.ops import reverse_adjacency
from oracle import refcpu


def _brute(nbr, deg):
    n, k = nbr.shape
    groups = [[] for _ in range(n)]
    for i in range(n):
        for e in range(k if deg is None else int(deg[i])):
            groups[int(nbr[i, e])].append(i * k + e)
    return groups


def test_reverse_adjacency_fixed_and_ragged():
    g = torch.Generator().manual_seed(0)
    n, k = 57, 7
    nbr = torch.randint(0, n, (n, k), generator=g, dtype=torch.int32)
    deg = torch.randint(0, k + 1, (n,), generator=g, dtype=torch.int32)
    for d in (None, deg):
        tab = nbr.clone()
        if d is not None:
            tab[torch.arange(k)[None, :] >= d[:, None]] = -1      # padding slots
        off, edge = reverse_adjacency(tab, d)
        assert off.dtype == torch.int64 and edge.dtype == torch.int64 and off.shape == (n + 1,)
        want = _brute(tab, d)
        for j in range(n):
            assert edge[off[j]:off[j + 1]].tolist() == want[j]   # stable: target order


def test_reverse_adjacency_rejects_out_of_range_sources():
    nbr = torch.tensor([[1, 5]], dtype=torch.int32)
    try:
        reverse_adjacency(nbr)
    except ValueError:
        return
    raise AssertionError("expected ValueError")


def test_oracle_train_batchnorm_updates_running_stats():
    torch.manual_seed(0)
    bn = torch.nn.BatchNorm1d(8).double().train()
    sd = {k: v.clone() for k, v in bn.state_dict().items()}
    x = torch.randn(40, 8, dtype=torch.float64)
    want = bn(x)
    got = refcpu._bn(sd, "", x, train=True) if False else refcpu.F.batch_norm(
        x, sd["running_mean"], sd["running_var"], sd["weight"], sd["bias"], True, 0.1, 1e-5)
    assert torch.allclose(got, want)
    sd2 = {"p.running_mean": torch.zeros(8, dtype=torch.float64),
           "p.running_var": torch.ones(8, dtype=torch.float64),
           "p.weight": bn.weight.detach().clone(), "p.bias": bn.bias.detach().clone()}
    out = refcpu._bn(sd2, "p", x, train=True)
    assert torch.allclose(out, want)
    assert torch.allclose(sd2["p.running_mean"], bn.running_mean)
    assert torch.allclose(sd2["p.running_var"], bn.running_var)
