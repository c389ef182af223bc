"""Multi-GPU mixing: simulated nodes sharded across GPUs, cross-shard edges carried by RCCL.

One process per GPU (torch.distributed, backend "nccl" = RCCL over xGMI).  The path shards
naturally: every output row depends only on the pre-round rows of its in-neighbours, so one
exchange per round suffices.

ShardPlan (pure host logic, identical on every rank — no plan exchange):
  * clique-aligned partition: whole cliques (topology['cliques']) go to ranks as contiguous runs,
    balanced by node count; without cliques, contiguous rank ranges;
  * rank r's local rows = its nodes (clique-contiguous order), followed by its HALO rows: every
    remote node some local row reads, grouped by owner rank (ascending global id within a group);
  * the local CSR keeps each row's operand order and weights and only renumbers columns, so the
    exact kernel on a shard returns the same bits as the single-GPU run.
ShardedMixer (one round):
  slabs are window-blocked [K, rows_in, w] so that each column window's halo block is contiguous
  (RCCL sends/receives contiguous buffers).  For window k: pack the rows peers need
  (index_select) and grouped isend/irecv (batch_isend_irecv) on a comm stream; the compute stream
  waits only for window k's exchange, then mixes it — so window k+1's exchange over xGMI overlaps
  window k's HBM-bound kernel.
The same code runs on gloo with CPU tensors and a CPU local-compute callable (tests, world size 2).
"""
import numpy as np
import torch
import torch.distributed as dist

from .topology import MixCSR


class LocalShard:
    def __init__(self, rank, nodes, halo, halo_owner, csr, cliques, send):
        self.rank = rank
        self.nodes = nodes            # global ids of local rows, local order
        self.halo = halo              # global ids of halo rows (grouped by owner)
        self.halo_owner = halo_owner  # owner rank of each halo row
        self.csr = csr                # MixCSR over local rows, n_in = n_local + n_halo
        self.cliques = cliques        # local cliques (local indices) or None
        self.send = send              # {peer: local indices peer needs, in peer's halo order}

    @property
    def n_local(self):
        return len(self.nodes)

    @property
    def rows_in(self):
        return len(self.nodes) + len(self.halo)

    def recv_ranges(self):
        """{peer: (first halo row, count)} — contiguous per owner."""
        out = {}
        for q in np.unique(self.halo_owner):
            idx = np.nonzero(self.halo_owner == q)[0]
            out[int(q)] = (self.n_local + int(idx[0]), len(idx))
        return out


class ShardPlan:
    def __init__(self, csr, cliques, world):
        n = csr.n
        if cliques:
            groups = [list(c) for c in cliques]
        else:
            groups = [[i] for i in range(n)]
        sizes = np.asarray([len(c) for c in groups])
        # contiguous runs of groups, balanced by node count
        cuts = np.searchsorted(np.cumsum(sizes), np.arange(1, world) * n / world, side="left")
        cuts = np.concatenate([[0], np.minimum(cuts + 1, len(groups)), [len(groups)]]).astype(int)
        cuts = np.maximum.accumulate(cuts)
        self.world = world
        self.csr = csr
        self.groups_of = [groups[cuts[r]:cuts[r + 1]] for r in range(world)]
        self.owner = np.empty(n, np.int64)
        self.local_index = np.empty(n, np.int64)
        self.nodes_of = []
        for r in range(world):
            nodes = [v for c in self.groups_of[r] for v in c]
            self.nodes_of.append(np.asarray(nodes, np.int64))
            self.owner[nodes] = r
            self.local_index[nodes] = np.arange(len(nodes))
        self.has_cliques = bool(cliques)
        self._halo = [self._halo_of(r) for r in range(world)]

    def _halo_of(self, r):
        rp, col = self.csr.row_ptr, self.csr.col
        nodes = self.nodes_of[r]
        need = set()
        for g in nodes:
            need.update(int(c) for c in col[rp[g]:rp[g + 1]] if self.owner[c] != r)
        halo = sorted(need, key=lambda v: (self.owner[v], v))
        return np.asarray(halo, np.int64)

    def local(self, r):
        nodes = self.nodes_of[r]
        halo = self._halo[r]
        halo_owner = self.owner[halo] if len(halo) else np.zeros(0, np.int64)
        nl = len(nodes)
        remap = {int(g): nl + i for i, g in enumerate(halo)}
        rp, col, val = self.csr.row_ptr, self.csr.col, self.csr.val
        counts, cols, vals = [], [], []
        for g in nodes:
            c = col[rp[g]:rp[g + 1]]
            cols.append(np.asarray([self.local_index[v] if self.owner[v] == r else remap[int(v)]
                                    for v in c], np.int64))
            vals.append(val[rp[g]:rp[g + 1]])
            counts.append(len(c))
        row_ptr = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
        lcsr = MixCSR(row_ptr, np.concatenate(cols).astype(np.int32) if cols else np.zeros(0, np.int32),
                      np.concatenate(vals).astype(np.float32) if vals else np.zeros(0, np.float32),
                      n_in=nl + len(halo)).validate()
        cliques = None
        if self.has_cliques:
            cliques = [[int(self.local_index[v]) for v in c] for c in self.groups_of[r]]
        send = {}
        for q in range(self.world):
            if q == r:
                continue
            h = self._halo[q]
            mine = h[self.owner[h] == r] if len(h) else h
            if len(mine):
                send[q] = self.local_index[mine]
        return LocalShard(r, nodes, halo, halo_owner, lcsr, cliques, send)


class DistTransport:
    """Halo exchange over torch.distributed point-to-point (RCCL on GPUs, gloo on CPU): per window,
    one grouped batch_isend_irecv with every peer."""

    def __init__(self, group=None):
        self.group = group

    def exchange(self, sm, k, xk):
        ops = []
        for q in sorted(set(sm.send_idx) | set(sm.recv)):
            if q in sm.send_idx:
                sb = sm.send_buf[q][k]
                torch.index_select(xk[:sm.n_local], 0, sm.send_idx[q], out=sb)
                ops.append(dist.P2POp(dist.isend, sb, q, group=self.group))
            if q in sm.recv:
                r0, cnt = sm.recv[q]
                ops.append(dist.P2POp(dist.irecv, xk[r0:r0 + cnt], q, group=self.group))
        return dist.batch_isend_irecv(ops) if ops else []

    @staticmethod
    def wait(handle):
        for wk in handle:
            wk.wait()                          # NCCL: the current stream waits, not the host


class LoopbackTransport:
    """Single-process stand-in for the RCCL exchange (tests on one GPU): every rank's ShardedMixer
    lives in this process; before a round the caller sets `inputs[rank]` to each rank's input slab
    and the exchange copies the rows a rank needs straight out of its peers' slabs."""

    def __init__(self):
        self.peers = {}
        self.inputs = {}

    def exchange(self, sm, k, xk):
        for q, (r0, cnt) in sorted(sm.recv.items()):
            peer = self.peers[q]
            src = self.inputs[q][k][:peer.n_local]
            xk[r0:r0 + cnt].copy_(src.index_select(0, peer.send_idx[sm.rank]))
        ev = torch.cuda.Event() if xk.is_cuda else None
        if ev is not None:
            ev.record(torch.cuda.current_stream(xk.device))
        return ev

    @staticmethod
    def wait(handle):
        if handle is not None:
            torch.cuda.current_stream().wait_event(handle)


def window_layout(p, windows):
    """(K, w): K column windows of w columns (w multiple of 256 so every window stays aligned)."""
    k = max(1, min(windows, (p + 255) // 256))
    w = ((p + k - 1) // k + 255) // 256 * 256
    k = (p + w - 1) // w
    return k, w


class ShardedMixer:
    """One rank's part of the round: exchange halo rows, mix local rows.

    x, out: window-blocked slabs [K, rows_in, w] (see empty()); columns >= p of the last window are
    padding.  compute(x2d, out2d, kernel) defaults to this rank's Mixer on its GPU."""

    def __init__(self, csr, cliques, world, rank, device, p, windows=8, group=None, compute=None,
                 transport=None):
        self.plan = ShardPlan(csr, cliques, world)
        self.shard = self.plan.local(rank)
        self.world, self.rank, self.group = world, rank, group
        self.device = torch.device(device)
        self.n_total = csr.n
        self.n_local = self.shard.n_local
        self.rows_in = self.shard.rows_in
        self.p = p
        self.k, self.w = window_layout(p, windows)
        if compute is None:
            from .ops import Mixer
            self.mixer = Mixer(csr=self.shard.csr, cliques=self.shard.cliques, device=self.device)
            compute = self._gpu_compute
        self.compute = compute
        self.recv = self.shard.recv_ranges()
        self.send_idx = {q: torch.from_numpy(np.asarray(v, np.int64)).to(self.device)
                         for q, v in self.shard.send.items()}
        # one send buffer per (peer, window): a window's buffer is rewritten only in the next round,
        # after this round's compute of that window has waited for its transfer
        self.send_buf = {q: [torch.empty((len(v), self.w), dtype=torch.float32, device=self.device)
                             for _ in range(self.k)] for q, v in self.shard.send.items()}
        self.halo_rows = len(self.shard.halo)
        self.is_cuda = self.device.type == "cuda"
        self.comm_stream = torch.cuda.Stream(self.device) if self.is_cuda else None
        self.transport = transport if transport is not None else DistTransport(group)
        if isinstance(self.transport, LoopbackTransport):
            self.transport.peers[rank] = self
        elif world > 1:
            dist.barrier(group=group)   # first collective: every rank joins before any P2P

    @classmethod
    def dcliques(cls, n_per_rank, clique_size, world, rank, interclique, device, p, seed=1337,
                 windows=8, group=None):
        from .generate import dcliques_csr
        csr, cliques = dcliques_csr(n_per_rank * world, clique_size, interclique, seed)
        return cls(csr, cliques, world, rank, device, p, windows=windows, group=group)

    def empty(self):
        return torch.empty((self.k, self.rows_in, self.w), dtype=torch.float32, device=self.device)

    def kernel_for(self, mode="fast", x=None):
        if hasattr(self, "mixer"):
            probe = x[0] if x is not None and x.dim() == 3 else x
            return self.mixer.kernel_for(mode, probe)
        return "cpu"

    def _gpu_compute(self, x2d, out2d, kernel=None, mode="fast"):
        self.mixer(x2d, out=out2d, kernel=kernel, mode=mode)

    def __call__(self, x, out, kernel=None, mode="fast", events=None):
        assert x.shape == (self.k, self.rows_in, self.w) and out.shape == x.shape
        cur = torch.cuda.current_stream(self.device) if self.is_cuda else None
        if events is not None:
            events[0].record(cur)
        if self.is_cuda:
            self.comm_stream.wait_stream(cur)     # x is final (previous round / initial fill)
        pending = []
        for k in range(self.k):
            if self.world > 1:
                if self.is_cuda:
                    with torch.cuda.stream(self.comm_stream):
                        pending.append(self.transport.exchange(self, k, x[k]))
                else:
                    pending.append(self.transport.exchange(self, k, x[k]))
            else:
                pending.append(None)
        for k in range(self.k):
            if pending[k] is not None:
                self.transport.wait(pending[k])
            cw = min(self.w, self.p - k * self.w)
            self.compute(x[k][:, :cw], out[k][:self.n_local, :cw], kernel=kernel, mode=mode)
        if events is not None:
            events[1].record(cur)
        return out
