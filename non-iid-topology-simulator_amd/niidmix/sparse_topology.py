#!/usr/bin/env python
"""Sparse topology writer: the reference's topology generator CLIs, emitting
the weights as a CSR (topology.csr.npz) instead of a dense N x N matrix inside topology.json.

    python -m niidmix.sparse_topology d-cliques    [--rundir R] [--interclique fully-connected]
                                                   [--max-clique-size 30] [--remove-clique-edges 0]
    python -m niidmix.sparse_topology random-graph [--rundir R] [--nb-neighbours 10] [--randomize]

Same arguments, defaults and params.json 'topology' section as the reference CLIs
(tools/setup/topology/d_cliques/random_cliques.py:38-80, tools/setup/topology/random_graph.py:54-83),
same graph (niidmix.generate restates the generators with the same RNG order; tests pin it), same
Metropolis-Hastings weights bit for bit (niidmix.topology.mh_csr), but O(N * degree) memory for
the weights (the fp32 diagonal is still reduced over dense rows, O(N^2) adds in batches, for bitwise
equality with weights.py:25): a 10 000-node d-cliques topology is ~12 MB of CSR instead of a ~1 GB JSON of
a dense matrix.  It also writes a topology.json that the reference's own loader reads unchanged
(setup.topology.load, called by the unchanged run.py:92-93): 'edges' and 'cliques' as the
reference writes them, 'weights': [] (an empty tensor once loaded) and 'weights-kind' /
'weights-csr' naming the Metropolis-Hastings CSR next to it; the plugin (niidmix.d_sgd) mixes
such a topology through niidmix.topology.to_csr, bit for bit the dense round.  The rundir's
nodes.json gives N, params.json 'meta' the seed, as in the reference.  Like the reference CLIs it
prints the rundir for the next pipeline stage when --rundir is not given.
"""
import argparse
import logging

from . import meta as m
from .generate import dcliques_csr, random_graph_csr
from .topology import write_sparse


def _nodes(rundir):
    nodes = m.load(rundir, "nodes.json")
    n = len(nodes)
    assert [nd["rank"] for nd in nodes] == list(range(n)), "nodes.json must list ranks 0..N-1 in order"
    return n


def d_cliques(args, rundir):
    params = m.params(rundir)
    n = _nodes(rundir)
    section = {"name": "d-cliques/random-cliques", "weights": args.weights,
               "interclique-topology": args.interclique,
               "max-clique-size": args.max_clique_size,
               "remove-clique-edges": args.remove_clique_edges}
    m.extend(rundir, "topology", section)
    seed = params["meta"]["seed"]
    nb_classes = params.get("dataset", {}).get("nb-classes", 10)
    if args.interclique == "fractal" and nb_classes != 10:
        raise SystemExit("fractal interclique: only the 10-class grouping is restated")
    csr, cliques = dcliques_csr(n, args.max_clique_size, args.interclique, seed,
                                args.remove_clique_edges)
    write_sparse(rundir, csr, cliques=cliques)
    logging.info("d-cliques: %d nodes, %d cliques, nnz %d", n, len(cliques), csr.nnz)


def random_graph(args, rundir):
    params = m.params(rundir)
    n = _nodes(rundir)
    section = {"name": "random-graph", "nb-neighbours": args.nb_neighbours,
               "weights": args.weights, "randomize": args.randomize,
               "topology-seed": params["meta"]["seed"]}
    m.extend(rundir, "topology", section)
    csr, _ = random_graph_csr(n, args.nb_neighbours, section["topology-seed"])
    write_sparse(rundir, csr)
    logging.info("random-graph: %d nodes, nnz %d", n, csr.nnz)


def main(argv=None):
    ap = argparse.ArgumentParser(description="Generate a topology with sparse weights (topology.csr.npz + a sparse topology.json).")
    sub = ap.add_subparsers(dest="kind", required=True)
    dc = sub.add_parser("d-cliques", help="random_cliques.py equivalent")
    dc.add_argument("--rundir", type=str, default=None)
    dc.add_argument("--interclique", type=str, default="fully-connected",
                    choices=["ring", "fractal", "smallworld", "fully-connected"])
    dc.add_argument("--weights", type=str, default="metropolis-hasting",
                    choices=["metropolis-hasting"])
    dc.add_argument("--max-clique-size", type=int, default=30)
    dc.add_argument("--remove-clique-edges", type=int, default=0)
    rg = sub.add_parser("random-graph", help="random_graph.py equivalent")
    rg.add_argument("--rundir", type=str, default=None)
    rg.add_argument("--weights", type=str, default="metropolis-hasting",
                    choices=["metropolis-hasting"])
    rg.add_argument("--nb-neighbours", type=int, default=10)
    rg.add_argument("--randomize", action="store_const", const=True, default=False)
    args = ap.parse_args(argv)
    rundir = m.rundir(args)
    log = m.params(rundir).get("meta", {}).get("log", "WARNING")
    logging.basicConfig(level=getattr(logging, str(log).upper(), None))
    (d_cliques if args.kind == "d-cliques" else random_graph)(args, rundir)
    if args.rundir is None:
        print(rundir)


if __name__ == "__main__":
    main()
