"""Gradient averaging on the GPU (k_grad_segment_mean, k_mix_csr | NIIDMIX_FLAG_MEAN) and the
drop-in niidmix.d_sgd.gradient against the golden fixtures produced by running the reference's
d_sgd.gradient (d_sgd.py:47-94): bit for bit, gradients and the parameters after the SGD step."""
import json

import numpy as np
import pytest
import torch

from conftest import grad_cases, load_grad

pytestmark = pytest.mark.gpu


class FlatModel(torch.nn.Module):
    def __init__(self, shapes):
        super().__init__()
        self.ps = torch.nn.ParameterList([torch.nn.Parameter(torch.zeros(s)) for s in shapes])


def _flat(nodes, attr):
    return np.stack([torch.cat([(q.grad if attr == "grad" else q).detach().reshape(-1)
                                for q in nd["model"].parameters()]).numpy() for nd in nodes])


def _nodes(d, params):
    from niidmix import d_sgd
    shapes = [tuple(s) for s in json.loads(str(d["shapes_json"]))]
    nodes = []
    for r in range(d["x"].shape[0]):
        m = FlatModel(shapes)
        off = 0
        with torch.no_grad():
            for q in m.parameters():
                k = q.numel()
                q.copy_(torch.from_numpy(d["x"][r, off:off + k].copy()).view_as(q))
                q.grad = torch.from_numpy(d["g"][r, off:off + k].copy()).view_as(q).clone()
                off += k
        nodes.append({"rank": r, "model": m, "optimizer": d_sgd.optimizer(m, params)})
    return nodes


@pytest.mark.parametrize("name", grad_cases())
def test_grad_mean_kernel_bitwise(name, gpu, oracle_mod):
    from niidmix.gradient import GradMean, build_grad_plan
    d, topo, params = load_grad(name)
    plan = build_grad_plan(d["g"].shape[0], topo, params)
    op = GradMean(plan, gpu)
    g = torch.from_numpy(d["g"]).to(gpu)
    out = op(g).cpu().numpy()
    stepped = np.zeros(plan.n, bool)
    stepped[plan.stepped] = True
    assert oracle_mod.bitwise_equal(out[stepped], d["g_out"][stepped]), name


@pytest.mark.parametrize("name", grad_cases())
def test_dsgd_gradient_dropin_bitwise(name, gpu, oracle_mod, monkeypatch):
    """niidmix.d_sgd.gradient(nodes, topology, params) == reference d_sgd.gradient: the averaged
    gradients and the stepped parameters, bit for bit, through the pinned gradient slab streamed in
    several column windows."""
    monkeypatch.setenv("NIIDMIX_WINDOW", "256")
    from niidmix import d_sgd
    d, topo, params = load_grad(name)
    nodes = _nodes(d, params)
    d_sgd.gradient(nodes, topo, params)
    from niidmix.gradient import build_grad_plan
    plan = build_grad_plan(len(nodes), topo, params)
    stepped = np.zeros(plan.n, bool)
    stepped[plan.stepped] = True
    assert oracle_mod.bitwise_equal(_flat(nodes, "grad")[stepped], d["g_out"][stepped]), name
    assert oracle_mod.bitwise_equal(_flat(nodes, "data"), d["y"]), name


def test_grad_segment_mean_strided_and_aliasing(gpu, oracle_mod):
    """A column window of a wider slab (ld > p, p % 4 != 0 -> scalar path) and the out-of-place
    check."""
    from niidmix import ops
    from niidmix.gradient import GradMean, build_grad_plan
    n = 64
    cliques = [list(range(i, n, 4)) for i in range(4)]
    plan = build_grad_plan(n, {"cliques": cliques, "edges": {}}, {"algorithm": {"clique-gradient": True}})
    op = GradMean(plan, gpu)
    gen = torch.Generator().manual_seed(0)
    full = torch.randn(n, 1000, generator=gen)
    g = full.to(gpu)[:, 3:3 + 517]
    out = torch.empty((n, 1024), device=gpu)[:, :517]
    op(g, out=out)
    ref = oracle_mod.grad_mean_c(full.numpy(), *_csr(plan), cols=(3, 520))[:, 3:520]
    assert oracle_mod.bitwise_equal(out.cpu().numpy(), ref)
    with pytest.raises(RuntimeError):
        ops.grad_segment_mean(g, op.seg_ptr, op.seg_row, g)


def _csr(plan):
    rows = [[r] for r in range(plan.n)]
    for s in range(len(plan.seg_ptr) - 1):
        seg = plan.seg_row[plan.seg_ptr[s]:plan.seg_ptr[s + 1]].tolist()
        for r in seg:
            rows[r] = seg
    return (np.cumsum([0] + [len(r) for r in rows]).astype(np.int64),
            np.asarray([c for r in rows for c in r], np.int32))


def test_grad_segment_mean_full_size(gpu, oracle_mod):
    """Headline shape (1000 nodes, 10 cliques of 100, P = 2^20): every member of a clique holds the
    same row, and sampled column windows equal the oracle bit for bit (columns are independent)."""
    from niidmix.generate import dcliques
    from niidmix.gradient import GradMean, build_grad_plan
    edges, cliques = dcliques(1000, 100, "fully-connected", seed=1337)
    plan = build_grad_plan(1000, {"cliques": cliques, "edges": edges},
                           {"algorithm": {"clique-gradient": True}})
    p = 1 << 20
    g = torch.empty((1000, p), device=gpu).normal_(generator=torch.Generator(gpu).manual_seed(0))
    out = GradMean(plan, gpu)(g)
    for c in cliques:
        rows = out[c]
        assert torch.equal(rows, rows[:1].expand_as(rows))
    row_ptr, col = _csr(plan)
    for c0 in (0, 12345, p - 64):
        win = g[:, c0:c0 + 64].cpu().numpy()
        ref = oracle_mod.grad_mean_c(win, row_ptr, col)
        assert oracle_mod.bitwise_equal(out[:, c0:c0 + 64].cpu().numpy(), ref)
