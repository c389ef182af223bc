"""D-Cliques topology generation for benchmarks and multi-GPU tests (support code, not the hot path).

The reference generates topologies offline (tools/setup/topology/d_cliques/random_cliques.py:18-37
and interclique.py:4-127).  The benchmark needs the same topology family at sizes the reference's
O(N^2) JSON path handles poorly (8 000 - 10 000 nodes), so this module restates those two
generators — same Python `random.Random` seeding and the same set/dict operations, hence the same
cliques and edge lists in the same order — and pairs them with the sparse MH builder
(topology.mh_csr).  tests/test_generate.py pins the restatement against the topologies the
reference itself produced (tests/golden/dcliques*.npz).
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


def dcliques(n, clique_size=100, interclique="fully-connected", seed=1337):
    """(edge lists {rank: list}, cliques) of a D-Cliques topology as random_cliques.py builds it."""
    cliques, intra = random_cliques(n, clique_size, seed)
    if interclique == "fully-connected":
        e = interclique_fully_connected(cliques, intra)
    elif interclique == "ring":
        e = interclique_ring(cliques, intra)
    elif interclique == "smallworld":
        e = interclique_smallworld(cliques, intra, seed)
    else:
        raise ValueError(f"unsupported interclique {interclique!r}")
    return {r: list(e[r]) for r in e}, cliques


def dcliques_csr(n, clique_size=100, interclique="fully-connected", seed=1337):
    edges, cliques = dcliques(n, clique_size, interclique, seed)
    return mh_csr(n, edges), cliques
