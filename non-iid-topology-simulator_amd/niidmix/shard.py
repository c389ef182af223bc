"""Multi-GPU mixing: two partitions of one round across GPUs (one process per GPU).

COLUMN STRIPES (StripedMixer, the default of bench.py --gpus N): the round is independent per
parameter column (Θ'[:, c] = Wᵀ Θ[:, c], d_sgd.py:96-116 mixes every tensor element-wise), so rank
r owns parameter columns [c0, c1) of EVERY node and mixes them with no exchange at all.  Results
are the single-GPU bits of those columns.  This is the natural split of the simulator, which
holds all nodes' models in one process.

NODE SHARDS (ShardedMixer): simulated nodes sharded across GPUs, cross-shard edges carried by
RCCL, for callers whose nodes' full parameter vectors must live on their own rank.

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
    def __init__(self, rank, nodes, halo, halo_owner, csr, cliques, send_block, send_shared,
                 recv):
        self.rank = rank
        self.nodes = nodes              # global ids of local rows, local order
        self.halo = halo                # global ids of halo rows (grouped by owner)
        self.halo_owner = halo_owner    # owner rank of each halo row
        self.csr = csr                  # MixCSR over local rows, n_in = n_local + n_halo
        self.cliques = cliques          # local cliques (local indices) or None
        self.send_block = send_block    # {peer: (a, b)}: local rows [a, b) only that peer reads
        self.send_shared = send_shared  # {peer: local indices of rows several peers read}
        self.recv = recv                # {peer: (first halo row, n_block, n_shared)}

    @property
    def n_local(self):
        return len(self.nodes)

    @property
    def rows_in(self):
        return len(self.nodes) + len(self.halo)

    @property
    def send(self):
        """{peer: every local index that peer reads, in the peer's halo order}."""
        out = {}
        for q in sorted(set(self.send_block) | set(self.send_shared)):
            a, b = self.send_block.get(q, (0, 0))
            out[q] = np.concatenate([np.arange(a, b), self.send_shared.get(q, np.zeros(0, np.int64))])
        return out


class ShardPlan:
    """Clique-aligned partition + halo plan, computed identically on every rank.

    Local row order of rank r: for each peer q (ascending) the rows ONLY q reads (a contiguous block:
    sent zero-copy, straight out of the slab), then rows several peers read (packed per peer), then
    interior rows.  The kernels address rows through the CSR / clique plan, so any order works;
    each row's operand order is unchanged (bit-exact)."""

    def __init__(self, csr, cliques, world):
        n = csr.n
        groups = [list(c) for c in cliques] if cliques else [[i] for i in range(n)]
        sizes = np.asarray([len(c) for c in groups])
        # contiguous runs of groups, balanced by node count
        cuts = np.searchsorted(np.cumsum(sizes), np.arange(1, world) * n / world, side="left")
        cuts = np.concatenate([[0], np.minimum(cuts + 1, len(groups)), [len(groups)]]).astype(int)
        cuts = np.maximum.accumulate(cuts)
        self.world = world
        self.csr = csr
        self.has_cliques = bool(cliques)
        self.groups_of = [groups[cuts[r]:cuts[r + 1]] for r in range(world)]
        self.owner = np.empty(n, np.int64)
        for r in range(world):
            for c in self.groups_of[r]:
                self.owner[c] = r
        rp, col = csr.row_ptr, csr.col
        # need[q]: remote rows rank q reads; readers[v]: ranks that read row v remotely
        self.need = [set() for _ in range(world)]
        dst_owner = np.repeat(self.owner, np.diff(rp))
        remote = self.owner[col] != dst_owner
        for q, v in zip(dst_owner[remote].tolist(), col[remote].tolist()):
            self.need[q].add(v)
        readers = {}
        for q in range(world):
            for v in self.need[q]:
                readers.setdefault(v, []).append(q)
        self.readers = readers
        self.local_index = np.empty(n, np.int64)
        self.nodes_of, self.blocks_of, self.shared_of = [], [], []
        for r in range(world):
            members = [v for c in self.groups_of[r] for v in c]
            excl = {q: [] for q in range(world)}
            shared, interior = [], []
            for v in members:
                rd = readers.get(v)
                if not rd:
                    interior.append(v)
                elif len(rd) == 1:
                    excl[rd[0]].append(v)
                else:
                    shared.append(v)
            order, blocks = [], {}
            for q in range(world):
                e = sorted(excl[q])
                if e:
                    blocks[q] = (len(order), len(order) + len(e))
                    order.extend(e)
            shared.sort()
            order.extend(shared)
            order.extend(interior)
            order = np.asarray(order, np.int64)
            self.local_index[order] = np.arange(len(order))
            self.nodes_of.append(order)
            self.blocks_of.append(blocks)
            self.shared_of.append(shared)

    def _halo_of(self, r):
        """Rows rank r reads remotely, grouped by owner: per owner q, q's block for r then the
        shared rows of q that r reads (both in q's local order)."""
        halo, owners, recv = [], [], {}
        start = 0
        for q in range(self.world):
            if q == r:
                continue
            a, b = self.blocks_of[q].get(r, (0, 0))
            blk = self.nodes_of[q][a:b].tolist()
            sh = [v for v in self.shared_of[q] if v in self.need[r]]
            sh.sort(key=lambda v: self.local_index[v])
            if blk or sh:
                recv[q] = (start, len(blk), len(sh))
                halo.extend(blk + sh)
                owners.extend([q] * (len(blk) + len(sh)))
                start += len(blk) + len(sh)
        return np.asarray(halo, np.int64), np.asarray(owners, np.int64), recv

    def local(self, r):
        nodes = self.nodes_of[r]
        halo, halo_owner, recv0 = self._halo_of(r)
        nl = len(nodes)
        recv = {q: (nl + s0, nb, ns) for q, (s0, nb, ns) in recv0.items()}
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
        send_shared = {}
        for q in range(self.world):
            if q == r:
                continue
            sh = [v for v in self.shared_of[r] if v in self.need[q]]
            if sh:
                send_shared[q] = np.asarray(sorted(self.local_index[v] for v in sh), np.int64)
        return LocalShard(r, nodes, halo, halo_owner, lcsr, cliques, dict(self.blocks_of[r]),
                          send_shared, recv)

    @property
    def _halo(self):
        return [self._halo_of(r)[0] for r in range(self.world)]


class _StagedHandle:
    """A gloo exchange of HIP tensors staged through host buffers (rehearsal only): the works, and
    the (host buffer, device rows) pairs to copy back once they completed."""

    def __init__(self, works, back):
        self.works, self.back = works, back


class DistTransport:
    """Halo exchange over torch.distributed point-to-point (RCCL on GPUs, gloo on CPU): per window,
    one grouped batch_isend_irecv with every peer.  A peer's exclusive rows go straight out of the
    slab (one contiguous block, no copy); rows several peers read are packed (index_select).

    With the gloo backend and HIP tensors (NIIDMIX_BENCH_BACKEND=gloo: several ranks rehearsing on
    one GPU, where RCCL refuses two ranks per device) every message is staged through host memory;
    the RCCL path never is."""

    def __init__(self, group=None):
        self.group = group

    def _staged(self, xk):
        return xk.is_cuda and dist.get_backend(self.group) == "gloo"

    def exchange(self, sm, k, xk):
        if self._staged(xk):
            return self._exchange_staged(sm, k, xk)
        ops = []
        sh = sm.shard
        for q in sorted(set(sh.send_block) | set(sh.send_shared) | set(sh.recv)):
            a, b = sh.send_block.get(q, (0, 0))
            if b > a:
                ops.append(dist.P2POp(dist.isend, xk[a:b], q, group=self.group))
            if q in sm.shared_idx:
                sb = sm.send_buf[q][k]
                torch.index_select(xk[:sm.n_local], 0, sm.shared_idx[q], out=sb)
                ops.append(dist.P2POp(dist.isend, sb, q, group=self.group))
            if q in sh.recv:
                r0, nb, ns = sh.recv[q]
                if nb:
                    ops.append(dist.P2POp(dist.irecv, xk[r0:r0 + nb], q, group=self.group))
                if ns:
                    ops.append(dist.P2POp(dist.irecv, xk[r0 + nb:r0 + nb + ns], q, group=self.group))
        return dist.batch_isend_irecv(ops) if ops else []

    def _exchange_staged(self, sm, k, xk):
        ops, back = [], []
        sh = sm.shard
        for q in sorted(set(sh.send_block) | set(sh.send_shared) | set(sh.recv)):
            a, b = sh.send_block.get(q, (0, 0))
            if b > a:
                ops.append(dist.P2POp(dist.isend, xk[a:b].cpu(), q, group=self.group))
            if q in sm.shared_idx:
                ops.append(dist.P2POp(dist.isend, torch.index_select(
                    xk[:sm.n_local], 0, sm.shared_idx[q]).cpu(), q, group=self.group))
            if q in sh.recv:
                r0, nb, ns = sh.recv[q]
                for a0, n0 in ((r0, nb), (r0 + nb, ns)):
                    if n0:
                        buf = torch.empty((n0, xk.shape[1]), dtype=xk.dtype)
                        ops.append(dist.P2POp(dist.irecv, buf, q, group=self.group))
                        back.append((buf, xk[a0:a0 + n0]))
        return _StagedHandle(dist.batch_isend_irecv(ops) if ops else [], back)

    @staticmethod
    def wait(handle):
        if isinstance(handle, _StagedHandle):
            for wk in handle.works:
                wk.wait()
            for buf, dst in handle.back:
                dst.copy_(buf)
            return
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
        for q, (r0, nb, ns) in sorted(sm.shard.recv.items()):
            peer = self.peers[q]
            src = self.inputs[q][k][:peer.n_local]
            idx = torch.from_numpy(peer.shard.send[sm.rank]).to(xk.device)
            xk[r0:r0 + nb + ns].copy_(src.index_select(0, idx))
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
        self.shared_idx = {q: torch.from_numpy(np.asarray(v, np.int64)).to(self.device)
                           for q, v in self.shard.send_shared.items()}
        # one pack buffer per (peer, window): a window's buffer is rewritten only in the next round,
        # after this round's compute of that window has waited for its transfer
        self.send_buf = {q: [torch.empty((len(v), self.w), dtype=torch.float32, device=self.device)
                             for _ in range(self.k)] for q, v in self.shard.send_shared.items()}
        self.halo_rows = len(self.shard.halo)
        self.is_cuda = self.device.type == "cuda"
        self.comm_stream = torch.cuda.Stream(self.device) if self.is_cuda else None
        self.transport = transport if transport is not None else DistTransport(group)
        if isinstance(self.transport, LoopbackTransport):
            self.transport.peers[rank] = self
        elif world > 1:
            dist.barrier(group=group)   # first collective: every rank joins before any P2P

    @classmethod
    def dcliques(cls, n_total, clique_size, world, rank, interclique, device, p, seed=1337,
                 windows=8, group=None):
        from .generate import dcliques_csr
        csr, cliques = dcliques_csr(n_total, clique_size, interclique, seed)
        return cls(csr, cliques, world, rank, device, p, windows=windows, group=group)

    @property
    def halo_bytes(self):
        """Bytes this rank receives per round (its halo rows x p fp32 columns)."""
        return self.halo_rows * self.p * 4

    @property
    def send_bytes(self):
        """Bytes this rank sends per round (every row some peer reads, once per reading peer)."""
        return sum(len(v) for v in self.shard.send.values()) * self.p * 4

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


def column_stripe(p, world, rank, align=1024):
    """Rank r's parameter columns [c0, c1): ceil(p / align) column units of `align` dealt as evenly
    as possible in rank order (stripes stay block-aligned for the column-blocked layout)."""
    if not 0 <= rank < world:
        raise ValueError(f"rank {rank} not in world of {world}")
    units = -(-p // align)
    base, extra = divmod(units, world)
    u0 = rank * base + min(rank, extra)
    u1 = u0 + base + (1 if rank < extra else 0)
    return min(u0 * align, p), min(u1 * align, p)


class StripedMixer:
    """One rank's column stripe of the round: every node, columns [c0, c1), no exchange.

    Fast mode keeps the stripe device-resident in the column-blocked layout (niidmix.memory) and
    runs the clique kernel; exact mode (or a topology without a clique plan) uses a row-major
    [N, c1 - c0] slab and the Mixer's kernel choice.  Either way the stripe's result is bitwise the
    single-GPU result's columns [c0, c1) (same kernel, same per-column arithmetic)."""

    def __init__(self, csr, cliques, world, rank, device, p, mode="fast", align=1024):
        from . import ops
        self.world, self.rank, self.p = world, rank, p
        self.device = torch.device(device)
        self.c0, self.c1 = column_stripe(p, world, rank, align)
        self.p_local = self.c1 - self.c0
        self.n_total = self.n_local = csr.n
        self.halo_rows = 0
        self.mode = mode
        self.mixer = ops.Mixer(csr=csr, cliques=cliques, device=self.device)
        # column-blocked stripes whenever the factored kernels read them (register tile up to 256
        # members, one-pass big-clique kernel up to 1024) and the plan has no cancelling terms, in
        # the device layout those kernels stream best (Mixer.device_layout: clique-contiguous rows,
        # block width per plan): node i lives at stripe row perm[i]
        self.blocked = (mode == "fast" and self.mixer.factored_safe and
                        self.mixer.plan.max_clique <= 1024 and self.p_local % 4 == 0)
        self.perm, self.block_cols = None, None
        if self.blocked:
            self.perm, self.block_cols = self.mixer.device_layout()
            self.mixer = self.mixer.relabeled(self.perm)

    @classmethod
    def dcliques(cls, n_total, clique_size, world, rank, interclique, device, p, seed=1337,
                 mode="fast"):
        from .generate import dcliques_csr
        csr, cliques = dcliques_csr(n_total, clique_size, interclique, seed)
        return cls(csr, cliques, world, rank, device, p, mode=mode)

    def empty(self):
        from . import memory
        if self.blocked:
            return memory.empty_blocked(self.n_total, self.p_local, self.device, self.block_cols)
        return memory.empty_slab(self.n_total, self.p_local, self.device)

    def to_layout(self, x):
        """This rank's stripe of a row-major [N, p_local] slab in rank order -> the device layout."""
        from . import memory
        if not self.blocked:
            out = self.empty()
            out.copy_(x)
            return out
        if self.perm is not None:
            rows = torch.empty_like(x)
            rows[torch.from_numpy(self.perm).to(x.device)] = x
            x = rows
        return memory.to_blocked(x, self.block_cols)

    def from_layout(self, y):
        """The device layout -> row-major [N, p_local] in rank order."""
        from . import memory
        if not self.blocked:
            return y
        y = memory.from_blocked(y, self.p_local)
        if self.perm is not None:
            y = y[torch.from_numpy(self.perm).to(y.device)]
        return y

    def kernel_for(self, mode="fast", x=None):
        return "clique" if self.blocked and mode == "fast" else self.mixer.kernel_for(mode)

    def __call__(self, x, out, kernel=None, mode=None, events=None):
        mode = mode or self.mode
        cur = torch.cuda.current_stream(self.device)
        if events is not None:
            events[0].record(cur)
        if self.blocked and mode == "fast":
            self.mixer.mix_blocked(x, out, self.p_local)
        else:
            self.mixer(x, out=out, kernel=kernel, mode=mode)
        if events is not None:
            events[1].record(cur)
        return out


class LocalShardedRound:
    """Node shards over several GPUs of THIS process (the simulator's own model, run.py:136)
    through the C-ABI sharded round (niidmix_mix_sharded_f32, include/niidmix.h): per round and
    shard, pack the rows peers read -> RCCL point-to-point halo exchange (one group over every
    shard; device-to-device copies when shards share a device) -> niidmix_mix_csr_f32 over
    [local rows | halo rows].  The ShardPlan and the RCCL communicators are built once per
    topology.  Exact mode is bitwise the single-GPU round (every row keeps its operand order).

    Slabs are ping-pong pairs per shard: round k reads xs[k % 2] and writes the local rows of
    xs[(k + 1) % 2]; scatter() fills the current input, gather() returns the current state."""

    def __init__(self, csr, cliques, devices, p):
        import ctypes
        from . import _lib
        self._lib = _lib
        self.devices = [torch.device(d) for d in devices]
        self.world = len(self.devices)
        self.p = p
        self.plan = ShardPlan(csr, cliques, self.world)
        self.shards = [self.plan.local(r) for r in range(self.world)]
        self.n_total = csr.n
        self._keep = []
        self.xs, self.bufs, self.streams, self.host = [], [], [], []
        self.cur = 0
        for r, (sh, dev) in enumerate(zip(self.shards, self.devices)):
            rows_in, nl = sh.rows_in, sh.n_local
            xs = [torch.zeros((max(rows_in, 1), p), dtype=torch.float32, device=dev) for _ in range(2)]
            peers = sorted(set(sh.send) | set(sh.recv))
            send = [np.asarray(sh.send.get(q, np.zeros(0, np.int64)), np.int64) for q in peers]
            send_ptr = np.concatenate([[0], np.cumsum([len(v) for v in send])]).astype(np.int64)
            send_rows = torch.from_numpy(np.concatenate(send).astype(np.int32) if send else
                                         np.zeros(0, np.int32)).to(dev)
            send_buf = torch.empty((max(int(send_ptr[-1]), 1), p), dtype=torch.float32, device=dev)
            recv_row = np.asarray([sh.recv[q][0] if q in sh.recv else nl for q in peers], np.int64)
            recv_cnt = np.asarray([sh.recv[q][1] + sh.recv[q][2] if q in sh.recv else 0
                                   for q in peers], np.int64)
            peer_arr = np.asarray(peers, np.int32)
            rp = torch.from_numpy(sh.csr.row_ptr).to(dev)
            cl = torch.from_numpy(sh.csr.col).to(dev)
            vl = torch.from_numpy(sh.csr.val).to(dev)
            self.xs.append(xs)
            self.bufs.append(send_buf)
            self.streams.append(torch.cuda.Stream(dev))
            host = dict(peer=peer_arr, send_ptr=send_ptr, recv_row=recv_row, recv_cnt=recv_cnt)
            self.host.append(host)
            self._keep += [rp, cl, vl, send_rows, peer_arr, send_ptr, recv_row, recv_cnt]
            host.update(rp=rp, cl=cl, vl=vl, send_rows=send_rows)
        dev_ids = (ctypes.c_int * self.world)(*[d.index if d.index is not None else 0
                                                for d in self.devices])
        h = ctypes.c_void_p()
        _lib.check(_lib.lib.niidmix_sharded_create(self.world, dev_ids, ctypes.byref(h)),
                   "niidmix_sharded_create")
        self.handle = h
        self.loopback = bool(_lib.lib.niidmix_sharded_is_loopback(h))

    def __del__(self):
        h = getattr(self, "handle", None)
        if h:
            self._lib.lib.niidmix_sharded_destroy(h)
            self.handle = None

    def _shard_structs(self):
        import ctypes
        from ._lib import ShardC
        arr = (ShardC * self.world)()
        a, b = self.cur, 1 - self.cur
        for r, (sh, hd) in enumerate(zip(self.shards, self.host)):
            c = arr[r]
            c.device = self.devices[r].index if self.devices[r].index is not None else 0
            c.n_peers = len(hd["peer"])
            c.n_local, c.rows_in = sh.n_local, sh.rows_in
            c.x, c.y = self.xs[r][a].data_ptr(), self.xs[r][b].data_ptr()
            c.row_ptr, c.col, c.val = hd["rp"].data_ptr(), hd["cl"].data_ptr(), hd["vl"].data_ptr()
            ptr = lambda v: v.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
            c.peer, c.send_ptr = ptr(hd["peer"]), ptr(hd["send_ptr"])
            c.send_rows = hd["send_rows"].data_ptr() if hd["send_rows"].numel() else None
            c.send_buf = self.bufs[r].data_ptr()
            c.recv_row, c.recv_count = ptr(hd["recv_row"]), ptr(hd["recv_cnt"])
            c.stream = self.streams[r].cuda_stream
        return arr

    def scatter(self, x):
        """x: the global [N, p] slab (rank order, any device) -> every shard's local input rows."""
        for r, sh in enumerate(self.shards):
            idx = torch.from_numpy(np.asarray(sh.nodes, np.int64)).to(x.device)
            self.xs[r][self.cur][:sh.n_local].copy_(x.index_select(0, idx))
        torch.cuda.synchronize()

    def gather(self):
        """The current global state [N, p] on the CPU, rank order."""
        torch.cuda.synchronize()
        out = torch.empty((self.n_total, self.p), dtype=torch.float32)
        for r, sh in enumerate(self.shards):
            out[torch.from_numpy(np.asarray(sh.nodes, np.int64))] = \
                self.xs[r][self.cur][:sh.n_local].cpu()
        return out

    def __call__(self, mode="exact"):
        """One round on every shard (enqueued on the shards' streams, after each device's current
        stream), then the roles of the two slabs swap."""
        from .ops import EXACT, FAST
        for r in range(self.world):
            self.streams[r].wait_stream(torch.cuda.current_stream(self.devices[r]))
        arr = self._shard_structs()
        rc = self._lib.lib.niidmix_mix_sharded_f32(self.handle, arr, self.p,
                                                   EXACT if mode == "exact" else FAST)
        self._lib.check(rc, "niidmix_mix_sharded_f32")
        for r in range(self.world):
            torch.cuda.current_stream(self.devices[r]).wait_stream(self.streams[r])
        self.cur = 1 - self.cur
