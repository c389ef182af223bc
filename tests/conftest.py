"""Test configuration.

Markers
  gpu   needs a real MI355X (run on the GPU box: python -m pytest tests -m gpu).  Everything else
        runs on the CPU-only development container (python -m pytest tests -m "not gpu").
The oracle (oracle/) is imported here as the CHECKER only.
"""
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_ROOT = os.path.join(REPO, "non-iid-topology-simulator_amd")
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (REPO, PKG_ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X GPU (HIP)")


def golden_cases(pattern=""):
    names = sorted(f[:-4] for f in os.listdir(GOLDEN) if f.endswith(".npz"))
    return [n for n in names if pattern in n and not n.startswith(("uniform_avg", "grad_", "consensus_", "logger_"))]


def grad_cases():
    """Gradient-averaging fixtures (tests/golden/grad_*.npz, d_sgd.gradient run by make_golden.py)."""
    return sorted(f[:-4] for f in os.listdir(GOLDEN) if f.startswith("grad_") and f.endswith(".npz"))


def load_grad(name):
    """(fixture arrays, topology with int keys as setup.topology.load returns it, params)."""
    import json
    d = np.load(os.path.join(GOLDEN, name + ".npz"))
    out = {k: d[k] for k in d.files}
    topo = json.loads(str(out["topology_json"]))
    topo["edges"] = {int(r): v for r, v in topo["edges"].items()}
    if "neighbourhoods" in topo:
        topo["neighbourhoods"] = {int(r): v for r, v in topo["neighbourhoods"].items()}
    params = json.loads(str(out["params_json"]))
    return out, topo, params


def load_golden(name):
    d = np.load(os.path.join(GOLDEN, name + ".npz"))
    out = {k: d[k] for k in d.files}
    if "cliques_flat" in out:
        f, p = out["cliques_flat"], out["cliques_ptr"]
        out["cliques"] = [f[p[i]:p[i + 1]].tolist() for i in range(len(p) - 1)]
    return out


@pytest.fixture(scope="session")
def oracle_mod():
    from oracle import oracle
    return oracle


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")
