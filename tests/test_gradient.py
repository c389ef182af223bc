"""Gradient averaging (--clique-gradient / --unbiased-gradient, d_sgd.py:47-94) on the CPU side:
the oracle restatement against the golden fixtures produced by running the reference's
d_sgd.gradient (tests/golden/make_golden.py), the plan builder that turns the topology into the
kernels' averaging lists, and the gradient slab's survival across training rounds."""
import json

import numpy as np
import pytest
import torch

from conftest import grad_cases, load_grad
from niidmix.gradient import build_grad_plan


def _segments_to_csr(plan):
    rows = [[r] for r in range(plan.n)]
    for s in range(len(plan.seg_ptr) - 1):
        seg = plan.seg_row[plan.seg_ptr[s]:plan.seg_ptr[s + 1]].tolist()
        for r in seg:
            rows[r] = seg
    row_ptr = np.cumsum([0] + [len(r) for r in rows]).astype(np.int64)
    return row_ptr, np.asarray([c for r in rows for c in r], np.int32)


def _plan_csr(plan):
    return _segments_to_csr(plan) if plan.seg_ptr is not None else (plan.row_ptr, plan.col)


@pytest.mark.parametrize("name", grad_cases())
def test_oracle_grad_mean_bitwise(name, oracle_mod):
    d, topo, params = load_grad(name)
    plan = build_grad_plan(d["g"].shape[0], topo, params)
    row_ptr, col = _plan_csr(plan)
    stepped = np.zeros(plan.n, bool)
    stepped[plan.stepped] = True
    y_np = oracle_mod.grad_mean_np(d["g"], row_ptr, col)
    y_c = oracle_mod.grad_mean_c(d["g"], row_ptr, col)
    assert oracle_mod.bitwise_equal(y_np[stepped], d["g_out"][stepped]), name
    assert oracle_mod.bitwise_equal(y_c, y_np), name
    # nodes the reference does not step keep their gradient
    assert oracle_mod.bitwise_equal(d["g_out"][~stepped], d["g"][~stepped])


@pytest.mark.parametrize("name", grad_cases())
def test_golden_step_is_sgd_of_mean(name, oracle_mod):
    """The fixture's parameters after gradient() are one torch SGD step (lr 0.1) with the averaged
    gradient on exactly the stepped nodes: the GPU drop-in only has to reproduce g_out."""
    d, topo, params = load_grad(name)
    plan = build_grad_plan(d["g"].shape[0], topo, params)
    x = torch.from_numpy(d["x"].copy())
    for r in plan.stepped:
        q = torch.nn.Parameter(x[r].clone())
        q.grad = torch.from_numpy(d["g_out"][r].copy())
        torch.optim.SGD([q], lr=0.1, momentum=0.0).step()
        x[r] = q.detach()
    assert oracle_mod.bitwise_equal(x.numpy(), d["y"]), name


def test_plan_kinds():
    topo = {"edges": {0: [1], 1: [0, 2], 2: [1, 3], 3: [2]}, "cliques": [[1, 0], [2, 3]]}
    p = build_grad_plan(4, topo, {"algorithm": {"clique-gradient": True}})
    assert p.kind == "clique" and p.seg_ptr.tolist() == [0, 2, 4] and p.seg_row.tolist() == [1, 0, 2, 3]
    assert p.stepped == [1, 0, 2, 3]
    # removed edges: node 2 no longer adjacent to 3 -> averages only itself; clique order kept
    topo_rm = {"edges": {0: [1], 1: [0, 2], 2: [1], 3: []}, "cliques": [[1, 0], [2, 3]]}
    p = build_grad_plan(4, topo_rm, {"algorithm": {"clique-gradient": True},
                                     "topology": {"remove-clique-edges": 1}})
    assert p.kind == "clique-removed"
    rows = [p.col[p.row_ptr[r]:p.row_ptr[r + 1]].tolist() for r in range(4)]
    assert rows == [[1, 0], [1, 0], [2], [3]]
    # a node in no clique: its own one-member segment, not stepped
    p = build_grad_plan(5, topo, {"algorithm": {"clique-gradient": True}})
    assert p.seg_row.tolist()[-1] == 4 and 4 not in p.stepped
    with pytest.raises(ValueError):
        build_grad_plan(4, {"cliques": [[0, 1], [1, 2]], "edges": {}}, {"algorithm": {"clique-gradient": True}})
    p = build_grad_plan(3, {"edges": {}, "neighbourhoods": {0: [2, 0], 1: [1], 2: [0, 1, 2]}},
                        {"algorithm": {"unbiased-gradient": True}})
    assert p.kind == "unbiased" and p.col.tolist() == [2, 0, 1, 0, 1, 2] and p.stepped == [0, 1, 2]
    assert build_grad_plan(3, {"edges": {}}, {"algorithm": {}}) is None


def test_grad_slab_survives_rounds():
    """NodeSlab(grads=True): .grad are views of the slab; zero_grad(set_to_none=False) + backward
    accumulates into the views (0 + g), so the slab stays the gradients' storage across rounds."""
    from niidmix.slab import NodeSlab
    torch.manual_seed(0)
    models = [torch.nn.Linear(5, 3) for _ in range(3)]
    opts = [torch.optim.SGD(m.parameters(), lr=0.1) for m in models]
    slab = NodeSlab(models, pin=False, grads=True)
    assert slab.host.shape == (3, 18) and float(slab.host.abs().sum()) == 0.0
    for _ in range(2):
        for m, o in zip(models, opts):
            o.zero_grad(set_to_none=False)
            m(torch.randn(4, 5)).sum().backward()
        assert slab.owns(models)
        for i, m in enumerate(models):
            flat = torch.cat([q.grad.reshape(-1) for q in m.parameters()])
            assert torch.equal(flat, slab.host[i])
