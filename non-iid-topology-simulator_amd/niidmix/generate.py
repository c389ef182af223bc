"""Topology generation restated for sparse ingestion, benchmarks and multi-GPU tests (support code,
not the hot path).

The reference generates topologies offline (tools/setup/topology/d_cliques/random_cliques.py:18-37
and interclique.py:4-127).  The benchmark needs the same topology family at sizes the reference's
O(N^2) JSON path handles poorly (8 000 - 10 000 nodes), so this module restates those two
generators — same Python `random.Random` seeding and the same set/dict operations, hence the same
cliques and edge lists in the same order — and pairs them with the sparse MH builder
(topology.mh_csr).  tests/test_generate.py pins the restatement against the topologies the
reference itself produced (tests/golden/dcliques*.npz).

random_graph / random_graph_csr restate setup/topology/random_graph.py:10-42 (the generator that
d_sgd.next_step re-runs every round under --randomize, d_sgd.py:223-234) the same way, so the
drop-in can rebuild a round's topology as a CSR in O(N * k) instead of the reference's dense N x N
compute_weights + JSON (tests/test_generate.py pins it against the reference-run randomgraph50
fixture and against the reference module itself where it is importable).
"""
import math
from random import Random

from .topology import mh_csr


def random_cliques(n, max_clique_size, seed):
    """random_cliques.cliques (random_cliques.py:18-37): draw cliques of max_clique_size from the
    remaining node set; the remainder forms the last clique.  Intra-clique edges: all pairs."""
    nodes = set(range(n))
    rand = Random()
    rand.seed(seed)
    cliques = []
    while len(nodes) > max_clique_size:
        c = rand.sample(tuple(nodes), max_clique_size)
        nodes.difference_update(c)
        cliques.append(list(c))
    cliques.append(list(nodes))
    edges = {}
    for c in cliques:
        members = set(c)
        for rank in members:
            edges[rank] = members.difference([rank])
    return cliques, edges


def _least_connected(clique):
    m = min(clique.values())
    return [k for k in clique.keys() if clique[k] <= m]


def interclique_fully_connected(cliques, edges):
    """interclique.fully_connected (interclique.py:57-75): one edge between every pair of cliques,
    attached to each clique's least-connected member (last in dict order)."""
    edges = {r: set(edges[r]) for r in edges}
    counts = [{k: 0 for k in c} for c in cliques]
    for i in range(len(counts) - 1):
        for j in range(i + 1, len(counts)):
            x = _least_connected(counts[i]).pop()
            counts[i][x] += 1
            y = _least_connected(counts[j]).pop()
            counts[j][y] += 1
            edges[x].add(y)
            edges[y].add(x)
    return edges


def interclique_ring(cliques, edges):
    """interclique.ring (interclique.py:4-18)."""
    cl = [set(c) for c in cliques]
    edges = {r: set(edges[r]) for r in edges}
    prev = cl[-1].pop() if len(cl[-1]) > 1 else list(cl[-1])[0]
    for clique in cl:
        current = clique.pop() if len(cl[-1]) > 1 else list(cl[-1])[0]
        edges[prev].add(current)
        edges[current].add(prev)
        prev = clique.pop()
    return edges


def interclique_smallworld(cliques, edges, seed):
    """interclique.smallworld (interclique.py:81-119): each clique links to cliques at ring offsets
    2^s (both directions, two per offset), preferring its least-connected members."""
    edges = {r: set(edges[r]) for r in edges}
    counts = [{k: 0 for k in c} for c in cliques]
    rand = Random()
    rand.seed(seed)

    def least(clique):
        m = min(clique.values())
        out = [k for k in clique.keys() if clique[k] == m]
        rand.shuffle(out)
        return out

    nc = len(counts)
    offsets = [2 ** s for s in range(0, math.ceil(math.log(nc) / math.log(2)))]
    for start in range(nc):
        for offset in offsets:
            for k in range(2):
                for sign in (-1, 1):
                    x = least(counts[start]).pop()
                    counts[start][x] += 1
                    c = (start + sign * (offset + k)) % nc
                    y = least(counts[c]).pop()
                    counts[c][y] += 1
                    edges[x].add(y)
                    edges[y].add(x)
    return edges


def interclique_fractal(cliques, edges, seed, nb_classes=10):
    """interclique.fractal (interclique.py:20-55): connect groups of nb_classes cliques pairwise
    (least-connected members, shuffled), merge each group into one, repeat until one remains."""
    edges = {r: set(edges[r]) for r in edges}
    groups = [{m: 0 for m in c} for c in cliques]
    rand = Random()
    rand.seed(seed)

    def least(clique):
        m = min(clique.values())
        lc = [k for k in clique.keys() if clique[k] <= m]
        rand.shuffle(lc)
        return lc

    def connect(cl):
        for i in range(len(cl) - 1):
            for j in range(i + 1, len(cl)):
                x = least(cl[i]).pop()
                cl[i][x] += 1
                y = least(cl[j]).pop()
                cl[j][y] += 1
                edges[x].add(y)
                edges[y].add(x)
        merged = {}
        for c in cl:
            merged.update(c)
        return merged

    while len(groups) > 1:
        toconnect = groups.copy()
        groups = [connect(toconnect[i:i + nb_classes]) for i in range(0, len(toconnect), nb_classes)]
    return edges


def remove_clique_edges(edges, cliques, k, seed):
    """d_cliques/utils.remove_clique_edges (utils.py:3-21): remove k random intra-clique edges per
    clique (all member pairs shuffled with one Random seeded once)."""
    rand = Random()
    rand.seed(seed)
    edges = {r: set(edges[r]) for r in edges}
    cliques = [list(c) for c in cliques]
    for clique in cliques:
        cand = [(clique[i], clique[j]) for i in range(len(clique) - 1)
                for j in range(i + 1, len(clique))]
        rand.shuffle(cand)
        for a, b in cand[:k]:
            edges[a].remove(b)
            edges[b].remove(a)
    return edges, cliques


def dcliques(n, clique_size=100, interclique="fully-connected", seed=1337, remove=0,
             nb_classes=10):
    """(edge lists {rank: list}, cliques) of a D-Cliques topology as random_cliques.py:38-80
    builds it (cliques, interclique edges, optional removed clique edges)."""
    cliques, intra = random_cliques(n, clique_size, seed)
    if interclique == "fully-connected":
        e = interclique_fully_connected(cliques, intra)
    elif interclique == "ring":
        e = interclique_ring(cliques, intra)
    elif interclique == "smallworld":
        e = interclique_smallworld(cliques, intra, seed)
    elif interclique == "fractal":
        e = interclique_fractal(cliques, intra, seed, nb_classes)
    else:
        raise ValueError(f"unsupported interclique {interclique!r}")
    if remove > 0:
        e, cliques = remove_clique_edges(e, cliques, remove, seed)
    return {r: list(e[r]) for r in e}, cliques


def dcliques_csr(n, clique_size=100, interclique="fully-connected", seed=1337, remove=0):
    edges, cliques = dcliques(n, clique_size, interclique, seed, remove)
    return mh_csr(n, edges), cliques


def random_graph(n, nb_neighbours, seed):
    """random_graph.create (random_graph.py:10-42): every node, in rank order, draws its missing
    neighbours from the shuffled list of nodes that still have room; retried until every node has
    exactly nb_neighbours.  Same Random seeding, list/set operations and insertion order as the
    reference, hence the same edge lists in the same (set iteration) order."""
    rand = Random()
    rand.seed(seed)
    count = 0
    while True:
        count += 1
        edges = {r: set() for r in range(n)}
        for rank in range(n):
            available = [m for m in range(n)
                         if m != rank and len(edges[m]) < nb_neighbours and m not in edges[rank]]
            rand.shuffle(available)
            toadd = nb_neighbours - len(edges[rank])
            for neighbour in available[:toadd]:
                edges[rank].add(neighbour)
                edges[neighbour].add(rank)
        if all(len(edges[r]) == nb_neighbours for r in range(n)):
            return {r: list(edges[r]) for r in edges}
        if count >= 1000:
            raise AssertionError("random_graph: could not find a working solution, aborting")


def random_graph_csr(n, nb_neighbours, seed):
    """(MixCSR with sparse MH weights, edge lists) of random_graph.generate_topology
    (random_graph.py:45-51) without the dense N x N weight matrix."""
    edges = random_graph(n, nb_neighbours, seed)
    return mh_csr(n, edges), edges
