"""Host-side mirror of the reference API (no GPU): module trees, state_dict keys,
parameter counts, construction semantics, and that there is no CPU fallback."""
import pytest
import torch

from mmpde_amd import (DMM, GraphCreator_FS_2D, ItpNet, MP_PDE_Solver_2D, burgers, cy)
from mmpde_amd.synth import build_models, cy_synth_mesh, generate_cy_mesh


def test_gnn_keys_and_counts():
    m = MP_PDE_Solver_2D(cy(ori_grid=torch.rand(10, 2)), time_window=1, eq_variables={})
    assert repr(m) == "GNN"
    keys = set(m.state_dict())
    # reference gnn_2d.py module tree; PyG BatchNorm wraps BatchNorm1d as `.module`
    for i in range(6):
        for sub in ("message_net_1.0", "message_net_2.0", "update_net_1.0", "update_net_2.0"):
            assert f"gnn_layers.{i}.{sub}.weight" in keys
        for b in ("weight", "bias", "running_mean", "running_var", "num_batches_tracked"):
            assert f"gnn_layers.{i}.norm.module.{b}" in keys
    for k in ("embedding_mlp.0.weight", "embedding_mlp.1.running_var", "embedding_mlp.3.bias",
              "embedding_mlp.4.weight", "output_mlp.0.weight", "output_mlp.2.weight",
              "output_mlp.4.bias"):
        assert k in keys
    assert m.gnn_layers[0].message_net_1[0].weight.shape == (128, 260)
    assert m.gnn_layers[0].update_net_1[0].weight.shape == (128, 257)
    assert sum(p.numel() for p in m.parameters()) == 616461


def test_dmm_keys_and_counts():
    grid = torch.rand(2521, 2)
    d = DMM(mode="graph", grid=grid, branch_layer=[4, 3], trunk_layer=[2, 16, 512],
            out_layer=[1024, 512, 1])
    assert sum(p.numel() for p in d.parameters()) == 2089938
    keys = set(d.state_dict())
    for k in ("trunk.fc0.weight", "out_nn.fc0.bias", "decoding_mlp.layers.1.weight",
              "output_mlp.4.weight", "gnn_layers.2.norm.module.running_mean",
              "embedding_mlp.4.running_var"):
        assert k in keys
    a = DMM(s=48, mode="array", branch_layer=7, trunk_layer=[2, 32, 512], out_layer=[1024, 512, 1])
    assert a.branch.fc2.weight.shape == (1024, 144)
    assert "branch.layers.3.weight" in a.state_dict()


def test_itpnet_keys():
    it = ItpNet(2521, None, [128, 64], [128, 64], [1, 4, 16, 4, 1])
    keys = set(it.state_dict())
    assert "layers.2.weight" in keys and "layers2.0.weight" in keys
    assert "layers3.5.weight" in keys                  # unused, kept for key parity
    assert it.down[6].weight.shape == (2521, 2048)
    ib = ItpNet(48, 48, [128, 64], [128, 64], [1, 4, 16, 4, 1])
    assert ib.down[6].weight.shape == (1, 4, 5, 5)


def test_no_cpu_fallback():
    pde, model, model_b, itp, dmm, gc = build_models("cy", grid=torch.rand(100, 2))
    class G:  # noqa: N801
        x = torch.zeros(100, 1)
        pos = torch.zeros(100, 3)
        nbr = torch.zeros(100, 35, dtype=torch.int32)
    with pytest.raises(RuntimeError):
        model(G())
    with pytest.raises(RuntimeError):
        dmm.mesh(torch.zeros(1, 100), torch.zeros(100, 2))
    with pytest.raises(RuntimeError):
        itp.res_cut(torch.zeros(1, 100))


def test_training_mode_needs_device_tensors():
    """train() mode runs the differentiable HIP path (tests/test_gpu_train.py);
    on host tensors it refuses instead of falling back to a CPU computation."""
    from mmpde_amd.graph import Data

    _, model, _, _, _, _ = build_models("cy", grid=torch.rand(100, 2), moving_mesh=False)
    model.train()
    g = Data(x=torch.rand(100, 1), edge_index=None)
    g.pos = torch.rand(100, 3)
    g.nbr = torch.zeros((100, 4), dtype=torch.int32)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        model(g)


def test_dmm_training_needs_device_tensors():
    """DMM training (mmpde_amd.dmm_train): the train()-mode DMM forward and the
    softmax smoother refuse host tensors; the samplers keep the reference's
    batch-size constraints (nu a multiple of 4 / 10) as errors."""
    from mmpde_amd import dmm_train as T

    _, _, _, _, dmm, _ = build_models("cy", grid=torch.rand(100, 2))
    dmm.train()
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        dmm(torch.zeros(1, 100), torch.rand(100, 2))
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        T.interpolate(torch.zeros(2, 8, 8), torch.rand(4, 1), torch.rand(4, 1))
    with pytest.raises(ValueError):
        T.sample_train_data(torch.zeros(5, 8, 8), 8, 6, "cpu")
    with pytest.raises(ValueError):
        T.sample_train_data_tri(torch.zeros(5, 100, 3), 8, 12, "cpu")


def test_pde_constants():
    c = cy(ori_grid=torch.zeros(3, 2))
    assert c.tmax == 2.9 and c.grid_size == (30, 2521) and abs(c.dt - 0.1) < 1e-12
    b = burgers()
    assert b.tmax == 30 and b.dt == 1.0 and b.movingmesh_grid_size == (31, 96, 96)


def test_create_data_and_grids():
    pde, _, _, _, _, gc = build_models("burgers", moving_mesh=False)
    u = torch.arange(3 * 31 * 4, dtype=torch.float32).reshape(3, 31, 4)
    d, l = gc.create_data(u, [1, 5, 30])
    assert torch.equal(d[1, 0], u[1, 4]) and torch.equal(l[2, 0], u[2, 30])
    t = gc.time_grid()
    assert t.shape == (31,) and float(t[-1]) == 30.0
    g = gc.uniform_grid("cpu")                       # 'ij': point p = i*48 + j
    assert torch.equal(g[1], torch.tensor([0.0, float(torch.linspace(0, 1, 48)[1])]))
    xi = gc.xi_grid_xy(48, 48, "cpu")                # np.meshgrid 'xy': p = j*48 + i
    assert xi[1, 1] == 0.0 and xi[48, 0] == 0.0 and xi[1, 0] > 0


def test_synth_mesh_fixture_reproducible():
    m = cy_synth_mesh()
    assert m.shape == (2521, 2)
    assert torch.equal(m, generate_cy_mesh())
    assert (((m[:, 0] - 0.25) ** 2 + (m[:, 1] - 0.5) ** 2) > 0.0025).all()


def test_graph_creator_signature():
    gc = GraphCreator_FS_2D(cy(ori_grid=torch.zeros(5, 2)), neighbors=35, connect_edge="knn",
                            time_window=1, t_resolution=30)
    assert gc.n == 35 and gc.tw == 1 and gc.t_res == 30 and gc.e == "knn"


def test_knn_policy_no_probe_during_capture(monkeypatch):
    """ops.KnnTablePolicy (the kNN table-or-scan choice of the rollout): a probe
    is never started inside a hipGraph capture, and a probe pending when a
    capture begins goes back to the full search instead of staying unresolved."""
    from mmpde_amd import ops

    pol = ops.KnnTablePolicy("cpu", 2, 100, ("graph",))
    st = pol.state["graph"]
    st["mode"], st["wait"] = "full", 0
    monkeypatch.setattr(ops, "_capturing", lambda: True)
    assert pol.use_table("graph") is False and pol.mode("graph") == "full"
    monkeypatch.setattr(ops, "_capturing", lambda: False)
    assert pol.use_table("graph") is True and pol.mode("graph") == "probe"
    # the probe's table call lands in a capture: no read-back can be queued
    monkeypatch.setattr(ops, "_capturing", lambda: True)
    pol.after_table("graph", None, 0)
    assert pol.mode("graph") == "full" and st["wait"] == ops.KnnTablePolicy.PROBE_EVERY
    assert st["pending"] is None
