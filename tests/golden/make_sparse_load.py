#!/usr/bin/env python
"""Fixture for the sparse-topology drop-in: what the REFERENCE loader makes of a rundir written by
`python -m niidmix.sparse_topology`.

Run in the development container only (it imports /root/reference; the GPU box never runs it):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_sparse_load.py

Steps:
  1. a rundir with nodes.json (300 ranks) and params.json (meta.seed 1337), then
     `niidmix.sparse_topology d-cliques --max-clique-size 30` into it (topology.csr.npz + a sparse
     topology.json: 'weights': []);
  2. the reference's own `setup.topology.load(rundir)` (tools/setup/topology/__init__.py:4-12,
     what the unchanged tools/simulate/run.py:92-93 calls) reads it;
  3. saved: the topology.json text the writer produced (sparse_dcliques300.written.json) and a
     summary of the loader's result (sparse_dcliques300.refload.json: weights type / dtype /
     shape, the int-keyed edges, cliques, the other keys).
Only data is stored; nothing from the reference is copied.
"""
import json
import os
import sys
import tempfile

REF = os.environ.get("NIID_REFERENCE", "/root/reference")
OUT = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(OUT))


def main():
    sys.path.insert(0, os.path.join(REPO, "non-iid-topology-simulator_amd"))
    from niidmix import sparse_topology
    with tempfile.TemporaryDirectory() as rd:
        with open(os.path.join(rd, "nodes.json"), "w") as f:
            json.dump([{"rank": r} for r in range(300)], f)
        with open(os.path.join(rd, "params.json"), "w") as f:
            json.dump({"meta": {"seed": 1337, "log": "WARNING"}, "dataset": {"nb-classes": 10}}, f)
        sparse_topology.main(["d-cliques", "--rundir", rd, "--max-clique-size", "30"])
        with open(os.path.join(rd, "topology.json")) as f:
            text = f.read()
        sys.path.insert(0, os.path.join(REF, "tools"))
        import importlib
        ref_topology = importlib.import_module("setup.topology")
        t = ref_topology.load(rd)
    w = t["weights"]
    summary = {
        "weights_type": type(w).__name__, "weights_dtype": str(w.dtype),
        "weights_shape": list(w.shape),
        "edges": {str(k): v for k, v in t["edges"].items()},
        "edge_key_types": sorted({type(k).__name__ for k in t["edges"]}),
        "cliques": t["cliques"],
        "keys": sorted(t.keys()),
        "extra": {k: t[k] for k in t if k not in ("edges", "weights", "cliques")},
    }
    with open(os.path.join(OUT, "sparse_dcliques300.written.json"), "w") as f:
        f.write(text)
    with open(os.path.join(OUT, "sparse_dcliques300.refload.json"), "w") as f:
        json.dump(summary, f)
    print("wrote sparse_dcliques300.written.json / .refload.json:", summary["weights_type"],
          summary["weights_dtype"], summary["weights_shape"], summary["keys"])


if __name__ == "__main__":
    main()
