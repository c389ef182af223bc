"""Drop-in host logic on CPU: NodeSlab views, meta/CLI registration."""
import json
import os
import sys

import torch

from niidmix import meta
from niidmix.slab import NodeSlab


def test_nodeslab_views_and_optimizer():
    torch.manual_seed(0)
    models = [torch.nn.Linear(7, 3) for _ in range(4)]
    before = [torch.cat([q.detach().reshape(-1).clone() for q in mm.parameters()]) for mm in models]
    opts = [torch.optim.SGD(mm.parameters(), lr=0.1) for mm in models]
    slab = NodeSlab(models, pin=False)
    assert slab.host.shape == (4, 7 * 3 + 3)
    for i in range(4):
        assert torch.equal(slab.host[i], before[i])
    # optimizer steps write straight into the slab
    x = torch.randn(5, 7)
    models[2](x).sum().backward()
    opts[2].step()
    flat = torch.cat([q.detach().reshape(-1) for q in models[2].parameters()])
    assert torch.equal(slab.host[2], flat)
    assert not torch.equal(slab.host[2], before[2])
    assert slab.owns(models) and not slab.owns(models[::-1])


def test_meta_extend_refuses_overwrite(tmp_path):
    d = str(tmp_path)
    meta.extend(d, "meta", {"seed": 1})
    assert meta.params(d, "meta") == {"seed": 1}
    try:
        meta.extend(d, "meta", {"seed": 2})
        raise RuntimeError("should have refused")
    except AssertionError:
        pass


def test_cli_registers_plugin(tmp_path):
    d = str(tmp_path)
    topo = {"edges": {"0": [1], "1": [0]}, "weights": [[0.5, 0.5], [0.5, 0.5]]}
    with open(os.path.join(d, "topology.json"), "w") as f:
        json.dump(topo, f)
    meta.extend(d, "topology", {"name": "ring"})
    from niidmix import d_sgd
    d_sgd.main(["--rundir", d, "--batch-size", "125"])
    alg = meta.params(d, "algorithm")
    assert alg["module"] == "niidmix.d_sgd" and alg["batch-size"] == 125
    assert alg["mixing-mode"] == "exact"


def test_blocked_layout_roundtrip_cpu():
    """niidmix.memory.to_blocked / from_blocked: [rows, p] <-> [ceil(p/B), rows, B]."""
    import torch
    from niidmix import memory
    x = torch.arange(5 * 9000, dtype=torch.float32).view(5, 9000)
    xb = memory.to_blocked(x, block_cols=4096)
    assert xb.shape == (3, 5, 4096)
    assert torch.equal(xb[1, 2, :10], x[2, 4096:4106])
    assert float(xb[2, :, 9000 - 8192:].abs().sum()) == 0.0
    assert torch.equal(memory.from_blocked(xb, 9000), x)


def test_mixing_devices_policy(monkeypatch):
    """One GPU per 64K parameter columns at most, NIIDMIX_DEVICES selects (no GPU needed)."""
    import torch
    from niidmix.slab import MIN_STRIPE_COLS, mixing_devices
    devs = [torch.device("cuda", i) for i in range(8)]
    assert mixing_devices(7850, devs) == devs[:1]                 # linear MNIST model
    assert mixing_devices(62006, devs) == devs[:1]                # LeNet size
    assert mixing_devices(1 << 20, devs) == devs                  # 1M parameters: all 8
    assert mixing_devices(3 * MIN_STRIPE_COLS, devs) == devs[:3]
    monkeypatch.setenv("NIIDMIX_DEVICES", "2,5")
    assert mixing_devices(1 << 20) == [torch.device("cuda", 2), torch.device("cuda", 5)]
