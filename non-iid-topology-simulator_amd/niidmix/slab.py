"""Host-resident node state for the drop-in.

The reference keeps every simulated node's model as its own nn.Module on the host between rounds
(training runs on CPU, d_sgd.py:186-213).  NodeSlab re-points the parameters of N identical models
at views of ONE pinned host slab [N, P] (row = node, flattened in model.parameters() order), so the
per-round mixing needs no gather/scatter: the slab streams to HBM, is mixed there by the HIP
kernels, and streams back.  Training, optimizers (the Parameter objects are unchanged, only their
.data) and the logger keep working on the models as before.

SlabMixer pipelines one round over column windows of the slab (columns are independent in Θ' = Wᵀ Θ):
    H2D window k+1  ||  mix window k  ||  D2H window k-1
on three HIP streams, so the round costs ~max(H2D, D2H) on PCIe rather than their sum.  The copies
are strided 2-D memcpys straight from/to the pinned slab (niidmix_copy2d_async).  Jacobi holds:
window k's inputs are on the device before its outputs are written back, and windows never share
columns.
"""
import ctypes
import os
import time

import torch

from . import _lib


def _flat_shapes(model):
    return [(p.shape, p.numel()) for p in model.parameters()]


class NodeSlab:
    """Parameters of `models` as views into one fp32 [N, P] host slab (pinned by default).

    grads=True backs the parameters' .grad tensors instead (the gradient slab of --clique-gradient /
    --unbiased-gradient, niidmix.gradient): each p.grad becomes a view of the slab, initialised from
    the current gradient (zeros where there is none).  The views survive training rounds as long as
    gradients are zeroed in place (optimizer.zero_grad(set_to_none=False), the reference's torch
    1.7.1 behaviour): backward then accumulates into the existing .grad (0 + g).
    """

    def __init__(self, models, pin=True, grads=False):
        models = list(models)
        if not models:
            raise ValueError("NodeSlab needs at least one model")
        shapes = _flat_shapes(models[0])
        for m in models:
            if _flat_shapes(m) != shapes:
                raise ValueError("all node models must have the same parameter shapes")
            for q in m.parameters():
                if q.dtype != torch.float32:
                    raise ValueError("the mixing kernels are fp32; got a %s parameter" % q.dtype)
        self.models = models
        self.shapes = shapes
        self.grads = grads
        self.n = len(models)
        self.p = sum(k for _, k in shapes)
        pin = pin and torch.cuda.is_available()
        self.host = torch.empty((self.n, self.p), dtype=torch.float32, pin_memory=pin)
        # a parameter gets a tensor over its own stretch of the slab with a storage of its own
        # size (torch.from_numpy over a slice): pickle.dumps(model.state_dict()) -- the reference
        # logger, logger.py:139,254 -- and torch.save serialise a tensor's WHOLE storage, which for
        # a plain view would be the whole [N, P] slab per node
        arr = self.host.numpy()
        with torch.no_grad():
            for i, m in enumerate(models):
                off = 0
                for q, (shape, k) in zip(m.parameters(), shapes):
                    if grads:
                        view = self.host[i, off:off + k]
                        if q.grad is None:
                            view.zero_()
                        else:
                            view.copy_(q.grad.detach().reshape(-1))
                        q.grad = view.view(shape)
                    else:
                        view = torch.from_numpy(arr[i, off:off + k])
                        view.copy_(q.detach().reshape(-1))
                        q.data = view.view(shape)
                    off += k
        # per model: (owning module, name, parameter) of every parameter in parameters() order
        # (shared parameters once, at their first place), for owns()
        self._slots = []
        for m in models:
            seen, slots = set(), []
            for mod in m.modules():
                for name, q in mod._parameters.items():
                    if q is not None and id(q) not in seen:
                        seen.add(id(q))
                        slots.append((mod, name, q))
            self._slots.append(slots)
        if not grads:
            from .guard import tag_slab
            tag_slab(models, self)

    def version(self):
        """Sum of the parameters' in-place write counters (torch's _version): any write through the
        parameters (an optimizer step, p.add_ / copy_ under no_grad, load_state_dict) changes it;
        the D2H write-back and .data writes do not."""
        return sum(q._version for slots in self._slots for _, _, q in slots)

    def owns(self, models):
        """True iff `models` are exactly this slab's models, in order, still backed by it (reads
        only parameter identities: no read-guard wait, niidmix.guard)."""
        from .guard import suspended
        if len(models) != self.n:
            return False
        base = self.host.data_ptr()
        with suspended():
            for i, m in enumerate(models):
                if m is not self.models[i]:
                    return False
                # every parameter, not just the first: one handed to a torch.multiprocessing queue
                # is moved to shared memory on its own (storage per parameter), and one replaced
                # by a new Parameter object is no longer a slab row (no module walk: ~0.5 us per
                # parameter)
                ptr = base + i * self.p * 4
                for (mod, name, q), (_, k) in zip(self._slots[i], self.shapes):
                    t = q.grad if self.grads else q
                    if mod._parameters.get(name) is not q or t is None or t.data_ptr() != ptr:
                        return False
                    ptr += k * 4
        return True


def _copy2d(dst, dpitch, src, spitch, width, rows, kind, stream):
    rc = _lib.lib.niidmix_copy2d_async(dst, dpitch, src, spitch, width, rows, kind,
                                       ctypes.c_void_p(stream.cuda_stream))
    _lib.check(rc, "niidmix_copy2d_async")


class SlabMixer:
    """One mixing round of a host [N, P] slab through the GPU, pipelined over column windows."""

    def __init__(self, mixer, n, p, device, window=1 << 15):
        self.mixer = mixer
        self.n, self.p = n, p
        self.device = torch.device(device)
        self.window = max(256, (min(window, p) + 255) // 256 * 256)
        w = self.window
        self.dx = [torch.empty((n, w), dtype=torch.float32, device=self.device) for _ in range(2)]
        self.dy = [torch.empty((n, w), dtype=torch.float32, device=self.device) for _ in range(2)]
        self.s_h2d = torch.cuda.Stream(self.device)
        self.s_mix = torch.cuda.Stream(self.device)
        self.s_d2h = torch.cuda.Stream(self.device)
        self.last_timing = None

    def mix(self, host, mode="exact", kernel=None, timing=False):
        """host: pinned fp32 [N, P] (may be any row-major slab with stride(1) == 1)."""
        t0 = time.perf_counter()
        self.launch(host, mode=mode, kernel=kernel, timing=timing)
        self.wait()
        if timing:
            self.last_timing["round_s"] = time.perf_counter() - t0
        return host

    def launch(self, host, mode="exact", kernel=None, timing=False):
        """Enqueue the round (H2D / mix / D2H of every window) without waiting for it."""
        n, p, w = self.n, self.p, self.window
        assert host.shape == (n, p) and host.dtype == torch.float32 and host.stride(1) == 1
        ld_h = host.stride(0) * 4
        base = host.data_ptr()
        nwin = (p + w - 1) // w
        ev_in = [torch.cuda.Event() for _ in range(nwin)]
        ev_mix = [torch.cuda.Event() for _ in range(nwin)]
        ev_out = [torch.cuda.Event() for _ in range(nwin)]
        t_ev = None
        self._timing = timing
        if timing:
            t_ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            t_ev[0].record(self.s_h2d)
        self._t_ev, self._nwin = t_ev, nwin
        for k in range(nwin):
            c0 = k * w
            cw = min(w, p - c0)
            buf = k % 2
            with torch.cuda.stream(self.s_h2d):
                if k >= 2:
                    self.s_h2d.wait_event(ev_mix[k - 2])          # dx[buf] consumed
                _copy2d(self.dx[buf].data_ptr(), w * 4, base + c0 * 4, ld_h, cw * 4, n, 0,
                        self.s_h2d)
                ev_in[k].record(self.s_h2d)
            with torch.cuda.stream(self.s_mix):
                self.s_mix.wait_event(ev_in[k])
                if k >= 2:
                    self.s_mix.wait_event(ev_out[k - 2])          # dy[buf] drained
                self.mixer(self.dx[buf][:, :cw], out=self.dy[buf][:, :cw], mode=mode,
                           kernel=kernel)
                ev_mix[k].record(self.s_mix)
            with torch.cuda.stream(self.s_d2h):
                self.s_d2h.wait_event(ev_mix[k])
                _copy2d(base + c0 * 4, ld_h, self.dy[buf].data_ptr(), w * 4, cw * 4, n, 1,
                        self.s_d2h)
                ev_out[k].record(self.s_d2h)
        if timing:
            t_ev[1].record(self.s_d2h)

    def wait(self):
        self.s_d2h.synchronize()
        if self._timing:
            t_ev = self._t_ev
            self.last_timing = {"gpu_span_s": t_ev[0].elapsed_time(t_ev[1]) / 1e3,
                                "windows": self._nwin, "window_cols": self.window}


class FusedRoundRunner:
    """One drop-in round with gradient averaging, fused on the device:
    per column window, H2D of the parameter AND gradient slabs, then on the device
        gradient mean (GradMean)  ->  SGD step on the stepped rows  ->  mixing (Mixer)
    and D2H of the mixed parameters and of the averaged gradients.  The reference's equivalent is
    d_sgd.gradient (CPU mean + optimizer.step on every stepped node) followed by d_sgd.average; per
    window the arithmetic is the same, bit for bit, and columns are independent, so windows
    pipeline as in SlabMixer.  The averaged gradients are written back to the host gradient slab,
    where the reference leaves them until the next zero_grad (update_gradients, d_sgd.py:37-45);
    grad_writeback=False (NIIDMIX_GRAD_WRITEBACK=0) skips that D2H for callers that never read
    .grad between rounds (the round is then H2D-bound: 8.4 GB per headline round)."""

    def __init__(self, grad_op, step_rows, lr, mixer, n, p, device, window=1 << 15,
                 grad_writeback=None):
        self.grad_op = grad_op
        self.mixer = mixer
        self.n, self.p = n, p
        self.device = torch.device(device)
        self.neg_lr = -float(lr)
        self.rows = torch.as_tensor(step_rows, dtype=torch.int32).to(self.device)
        self.window = max(256, (min(window, p) + 255) // 256 * 256)
        w = self.window
        mk = lambda: torch.empty((n, w), dtype=torch.float32, device=self.device)  # noqa: E731
        self.dp = [mk(), mk()]
        self.dg = [mk(), mk()]
        self.dy = [mk(), mk()]
        self.dm = [mk(), mk()]
        if grad_writeback is None:
            grad_writeback = os.environ.get("NIIDMIX_GRAD_WRITEBACK", "1") != "0"
        self.grad_writeback = grad_writeback
        self.s_h2d = torch.cuda.Stream(self.device)
        self.s_mix = torch.cuda.Stream(self.device)
        self.s_d2h = torch.cuda.Stream(self.device)
        self.last_timing = None

    def run(self, host_params, host_grads, mode="exact", timing=False):
        t0 = time.perf_counter()
        self.launch(host_params, host_grads, mode=mode)
        self.wait()
        if timing:
            self.last_timing = {"round_s": time.perf_counter() - t0,
                                "windows": (self.p + self.window - 1) // self.window,
                                "window_cols": self.window}
        return host_params

    def launch(self, host_params, host_grads, mode="exact"):
        """Enqueue the fused round of every window without waiting for it."""
        from . import ops
        n, p, w = self.n, self.p, self.window
        for h in (host_params, host_grads):
            assert h.shape == (n, p) and h.dtype == torch.float32 and h.stride(1) == 1
        ld_p, ld_g = host_params.stride(0) * 4, host_grads.stride(0) * 4
        bp, bg = host_params.data_ptr(), host_grads.data_ptr()
        nwin = (p + w - 1) // w
        ev_in = [torch.cuda.Event() for _ in range(nwin)]
        ev_mix = [torch.cuda.Event() for _ in range(nwin)]
        ev_out = [torch.cuda.Event() for _ in range(nwin)]
        for k in range(nwin):
            c0 = k * w
            cw = min(w, p - c0)
            buf = k % 2
            with torch.cuda.stream(self.s_h2d):
                if k >= 2:
                    self.s_h2d.wait_event(ev_mix[k - 2])
                _copy2d(self.dp[buf].data_ptr(), w * 4, bp + c0 * 4, ld_p, cw * 4, n, 0, self.s_h2d)
                _copy2d(self.dg[buf].data_ptr(), w * 4, bg + c0 * 4, ld_g, cw * 4, n, 0, self.s_h2d)
                ev_in[k].record(self.s_h2d)
            with torch.cuda.stream(self.s_mix):
                self.s_mix.wait_event(ev_in[k])
                if k >= 2:
                    self.s_mix.wait_event(ev_out[k - 2])
                xp, xg, gm = self.dp[buf][:, :cw], self.dg[buf][:, :cw], self.dm[buf][:, :cw]
                self.grad_op(xg, out=gm)
                if self.rows.numel():
                    ops.sgd_step_rows(xp, gm, self.rows, self.neg_lr)
                self.mixer(xp, out=self.dy[buf][:, :cw], mode=mode)
                ev_mix[k].record(self.s_mix)
            with torch.cuda.stream(self.s_d2h):
                self.s_d2h.wait_event(ev_mix[k])
                _copy2d(bp + c0 * 4, ld_p, self.dy[buf].data_ptr(), w * 4, cw * 4, n, 1, self.s_d2h)
                if self.grad_writeback:
                    _copy2d(bg + c0 * 4, ld_g, self.dm[buf].data_ptr(), w * 4, cw * 4, n, 1,
                            self.s_d2h)
                ev_out[k].record(self.s_d2h)

    def wait(self):
        self.s_d2h.synchronize()


class SampleAverage:
    """The 'sample' topology's round as a per-window device op (d_sgd.py:235-250): the average of
    the active nodes' rows, setup.model.average(models, [1/k]*k) (model/__init__.py:15-25: exact
    CSR kernel, one output row, NIIDMIX_FLAG_AVERAGE_ONLY, weights fp32(1/k) in the sample's
    order), then update_models(all_models, avg) of EVERY row (d_sgd.py:29-35: k_update_rows).
    Callable like a Mixer, so SlabMixer / MultiDeviceRound stream the pinned slab through it: one
    H2D and one D2H of the slab per round, no host-side stacking or per-tensor CPU updates."""

    def __init__(self, device):
        self.device = torch.device(device)
        self.row_ptr = self.col = self.val = None
        self._avg = None

    def set_active(self, rows, weights):
        import numpy as np
        k = len(rows)
        if k == 0:
            raise ValueError("sample round with no active node")
        w = np.asarray([float(v) for v in weights], np.float64).astype(np.float32)
        self.row_ptr = torch.tensor([0, k], dtype=torch.int64, device=self.device)
        self.col = torch.tensor(list(rows), dtype=torch.int32, device=self.device)
        self.val = torch.from_numpy(w).to(self.device)

    def __call__(self, x, out=None, mode="exact", kernel=None):
        from . import ops
        if out is None:
            out = torch.empty_like(x)
        cols = x.shape[1]
        if self._avg is None or self._avg.shape[1] < cols:
            self._avg = torch.empty((1, cols), dtype=torch.float32, device=self.device)
        avg = self._avg[:, :cols]
        ops.mix_csr(x, self.row_ptr, self.col, self.val, avg, ops.EXACT | ops.AVERAGE_ONLY)
        ops.update_rows(x, avg[0], out)
        return out


# ------------------------------------------------------------------------------------------------
# several GPUs in ONE process (the simulator is one process, run.py:136)
MIN_STRIPE_COLS = 1 << 16


def mixing_devices(p, devices=None):
    """The devices a host-resident round of P columns is spread over: NIIDMIX_DEVICES
    ("0,1,2,3"), else every visible GPU, but at most one per MIN_STRIPE_COLS columns (a LeNet-size
    model stays on one GPU; a 1M-parameter model uses up to 16)."""
    if devices is None:
        env = os.environ.get("NIIDMIX_DEVICES")
        if env:
            devices = [torch.device("cuda", int(i)) for i in env.split(",") if i.strip()]
        else:
            devices = [torch.device("cuda", i) for i in range(torch.cuda.device_count())]
    devices = [torch.device(d) for d in devices]
    k = max(1, min(len(devices), -(-p // MIN_STRIPE_COLS)))
    return devices[:k]


class MultiDeviceRound:
    """One host-resident round spread over several GPUs of this process by parameter-column
    stripes (niidmix.shard.column_stripe: the round is independent per column, d_sgd.py:96-116
    mixes every tensor element-wise), with no exchange between the GPUs: each device runs its own
    window pipeline (its own streams, buffers and PCIe link) on its stripe of the pinned slab(s),
    all devices enqueued before any is waited for.

      make(device, n, cols) -> a runner with launch(*host_stripes, **kw) / wait()
                               (SlabMixer, FusedRoundRunner)
    Results are bitwise those of one device: same kernels, same per-column arithmetic."""

    def __init__(self, make, n, p, devices, align=1024):
        from .shard import column_stripe
        self.n, self.p = n, p
        self.devices = [torch.device(d) for d in devices]
        world = len(self.devices)
        self.stripes = [column_stripe(p, world, r, align) for r in range(world)]
        self.runners = []
        for dev, (c0, c1) in zip(self.devices, self.stripes):
            self.runners.append(make(dev, n, c1 - c0) if c1 > c0 else None)
        self.last_timing = None

    def run(self, *hosts, timing=False, **kw):
        t0 = time.perf_counter()
        for runner, (c0, c1) in zip(self.runners, self.stripes):
            if runner is not None:
                with torch.cuda.device(runner.device):
                    runner.launch(*[h[:, c0:c1] for h in hosts], **kw)
        for runner in self.runners:
            if runner is not None:
                runner.wait()
        if timing:
            self.last_timing = {"round_s": time.perf_counter() - t0,
                                "devices": [str(d) for d in self.devices],
                                "stripes": self.stripes}
        return hosts[0]


# ------------------------------------------------------------------------------------------------
# row-streamed round: the PCIe copies hidden behind the CPU part of the round
class ResidentRound:
    """The host-resident round with its PCIe traffic overlapped with the CPU part of the round
    (the reference's round is train every node -> optimizer.step() every node
    -> average, d_sgd.py:186-220).

    The host slabs (each device: its column stripe of every row) stay resident in HBM: `n_in`
    input buffers (the parameter slab; with gradient averaging also the gradient slab) and `n_out`
    output buffers.  Per round:
      row_ready(i)   node i's rows are final (its parameters right after its optimizer.step(),
                     d_sgd.py:51-52; its gradients right after its backward(), d_sgd.py:196):
                     once every row of i's block of `block` rows is final, the block goes H2D on
                     a copy stream while the CPU carries on with the next nodes;
      mix(mode)      after the last node: the remaining blocks go up, the device op runs (for the
                     plain round the Mixer: dx -> dy, the same bits as every other path), and the
                     outputs come back D2H block by block in row order, one event per block;
      wait_row(i)    the next round's training of node i waits only for its own block
                     (d_sgd.py:186-198 reads row i first); wait_all() for readers of every model.
    Jacobi holds: every H2D of a round precedes its op (stream order), and the next round's H2D
    into the inputs waits for this round's op.  Several GPUs: one column stripe each, as
    MultiDeviceRound (bitwise the one-GPU round).

      make_op(dev, part) -> op(ins, outs, mode, kernel)   the device op of one stripe
                            (part: the stripe's dict; ops may keep state in it)"""

    def __init__(self, make_op, n, p, devices, block=8, align=1024, n_in=1, n_out=1):
        from .shard import column_stripe
        self.n, self.p = n, p
        self.block = max(1, int(block))
        self.nblk = -(-n // self.block)
        self.n_in, self.n_out = n_in, n_out
        self.devices = [torch.device(d) for d in devices]
        world = len(self.devices)
        self.parts = []
        for r, dev in enumerate(self.devices):
            c0, c1 = column_stripe(p, world, r, align)
            if c1 <= c0:
                continue
            w = c1 - c0
            mk = lambda: torch.empty((n, w), dtype=torch.float32, device=dev)  # noqa: E731
            part = {"dev": dev, "c0": c0, "w": w,
                    "ins": [mk() for _ in range(n_in)], "outs": [mk() for _ in range(n_out)],
                    "s_h2d": torch.cuda.Stream(dev), "s_mix": torch.cuda.Stream(dev),
                    "s_d2h": torch.cuda.Stream(dev), "ev_mix": None}
            part["op"] = make_op(dev, part)
            self.parts.append(part)
        self.hosts = None
        self.hosts_out = None
        self._count = [0] * self.nblk      # rows of each block made final this round
        self._sent = [False] * self.nblk
        self._done = None                  # per block: the D2H events of the last op
        self._d2h_next = 0                 # row blocks whose D2H is enqueued (paced write-back)
        self._d2h_outs = []
        self._pace = 0
        # the device outputs (outs[0]: the mixed parameters) hold the models' current values: set
        # by mix(), cleared by begin() and by guarded writes (niidmix.guard); read by niidmix.logger
        # and the device-step round through current(), which also compares the models' version
        # counters (version_of: NodeSlab.version) with their value at mix() -- an in-place write
        # through a parameter (p.add_ under no_grad, an optimizer step) is caught there.  Writes
        # that bypass both (p.data.copy_, a raw pointer) are not: call
        # niidmix.d_sgd.invalidate(nodes) after such a write.
        self.fresh = False
        self.version_of = None
        self.models_version = None
        self.last_timing = None

    @staticmethod
    def fits(n, p, devices, buffers=2, frac=0.8):
        """Enough free HBM for the resident buffers on every device (else: windowed round)."""
        world = max(1, len(devices))
        need = buffers * n * (-(-p // world)) * 4
        for d in devices:
            free, _ = torch.cuda.mem_get_info(torch.device(d))
            if need > frac * free:
                return False
        return True

    @property
    def host(self):
        return None if self.hosts is None else self.hosts[0]

    def begin(self, *hosts, outs=None, resident_in0=False):
        """Start a round: `hosts` are the pinned [N, P] input slabs (n_in of them), `outs` the host
        slabs the outputs return to (default: the first n_out inputs).  Nothing is sent yet.

        resident_in0: input 0 is NOT sent; the device output 0 of the last round (which holds the
        models' current values: `fresh`) becomes this round's input 0 -- the two device buffers swap
        roles -- and hosts[0] must be None (the device-side SGD step of the parameters)."""
        assert len(hosts) == self.n_in
        self._enqueue_d2h(self.nblk)               # a paced write-back: the rest now (from the
        if resident_in0:                           # output buffers as they are before the swap)
            assert hosts[0] is None and self.current(), \
                "resident input 0 needs the last round's output"
            for pt in self.parts:
                pt["ins"][0], pt["outs"][0] = pt["outs"][0], pt["ins"][0]
        for h in hosts:
            assert h is None or (h.shape == (self.n, self.p) and h.dtype == torch.float32 and
                                 h.stride(1) == 1)
        self.hosts = list(hosts)
        outs = list(outs) if outs is not None else list(hosts[:self.n_out])
        assert len(outs) == self.n_out and all(h is not None for h in outs)
        self.hosts_out = outs
        self.fresh = False
        self._count = [0] * self.nblk
        self._sent = [False] * self.nblk
        for pt in self.parts:
            pt["s_h2d"].wait_stream(pt["s_d2h"])   # the host rows come back before they go up

    def _rows(self, b):
        r0 = b * self.block
        return r0, min(self.n, r0 + self.block) - r0

    def _h2d(self, b):
        r0, rows = self._rows(b)
        for pt in self.parts:
            s = pt["s_h2d"]
            if pt["ev_mix"] is not None:
                s.wait_event(pt["ev_mix"])         # the previous round's op has read the inputs
                pt["ev_mix"] = None
            w = pt["w"]
            for h, d in zip(self.hosts, pt["ins"]):
                if h is None:                      # resident input (begin(resident_in0=True))
                    continue
                _copy2d(d.data_ptr() + r0 * w * 4, w * 4,
                        h.data_ptr() + (r0 * h.stride(0) + pt["c0"]) * 4, h.stride(0) * 4, w * 4,
                        rows, 0, s)
        self._sent[b] = True

    def row_ready(self, i):
        """Row i of the input slabs is final for this round: send its block once it is complete."""
        if self.hosts is None:
            return
        b = i // self.block
        self._count[b] += 1
        if self._count[b] == self._rows(b)[1] and not self._sent[b]:
            self._h2d(b)

    def mix(self, mode="exact", kernel=None, timing=False):
        """Enqueue the rest of the round (remaining H2D, the device op, D2H by block); returns at
        once."""
        t0 = time.perf_counter()
        delay = int(os.environ.get("NIIDMIX_D2H_DELAY_CYCLES", "0"))
        self._enqueue_d2h(self.nblk)               # the previous round's paced write-back: all
        unsent = sum(1 for s in self._sent if not s)
        for b in range(self.nblk):
            if not self._sent[b]:
                self._h2d(b)
        done = [[] for _ in range(self.nblk)]
        t_ev = []
        for pt in self.parts:
            with torch.cuda.device(pt["dev"]):
                sm, sd = pt["s_mix"], pt["s_d2h"]
                sm.wait_stream(pt["s_h2d"])
                sm.wait_stream(sd)                  # outputs drained by the previous round's D2H
                if timing:
                    ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                    ev[0].record(sm)
                with torch.cuda.stream(sm):
                    pt["op"](pt["ins"], pt["outs"], mode, kernel)
                ev_mix = torch.cuda.Event()
                ev_mix.record(sm)
                pt["ev_mix"] = ev_mix
                if timing:
                    ev[1].record(sm)
                    t_ev.append(ev)
                sd.wait_event(ev_mix)
                if delay:                           # test knob: a late write-back (guard tests)
                    with torch.cuda.stream(sd):
                        torch.cuda._sleep(delay)
        self._done = done
        self._d2h_next = 0
        self._d2h_outs = list(self.hosts_out)
        # paced write-back (NIIDMIX_D2H_PACE = L > 0): only the first L row blocks go D2H now; the
        # rest follow as the next round's training reaches them (wait_row keeps L blocks ahead),
        # spreading the 4.2 GB of a headline round over the training instead of one ~85 ms burst
        # through the host's memory.  0 (default): every block now.
        pace = int(os.environ.get("NIIDMIX_D2H_PACE", "0"))
        self._enqueue_d2h(self.nblk if pace <= 0 else min(self.nblk, pace))
        self._pace = pace
        self.fresh = True
        self.models_version = self.version_of() if self.version_of is not None else None
        self.hosts = None                           # row_ready() is a no-op until begin()
        self._timing = (timing, t0, t_ev, unsent)

    def _enqueue_d2h(self, upto):
        """Enqueue the D2H of row blocks [_d2h_next, upto), one event per block and device."""
        if self._done is None or upto <= self._d2h_next:
            return
        for pt in self.parts:
            with torch.cuda.device(pt["dev"]):
                sd = pt["s_d2h"]
                w = pt["w"]
                for b in range(self._d2h_next, upto):
                    r0, rows = self._rows(b)
                    for h, d in zip(self._d2h_outs, pt["outs"]):
                        _copy2d(h.data_ptr() + (r0 * h.stride(0) + pt["c0"]) * 4, h.stride(0) * 4,
                                d.data_ptr() + r0 * w * 4, w * 4, w * 4, rows, 1, sd)
                    e = torch.cuda.Event()
                    e.record(sd)
                    self._done[b].append(e)
        self._d2h_next = upto

    def wait_row(self, i):
        """Block until row i's outputs are back in the host slabs."""
        if self._done is not None:
            b = i // self.block
            if self._d2h_next <= b:
                self._enqueue_d2h(min(self.nblk, b + max(self._pace, 1)))
            elif self._pace > 0:
                self._enqueue_d2h(min(self.nblk, b + self._pace))
            for e in self._done[b]:
                e.synchronize()

    def wait_all(self):
        if self._done is None:
            return
        self._enqueue_d2h(self.nblk)
        for evs in self._done:
            for e in evs:
                e.synchronize()
        timing, t0, t_ev, unsent = self._timing
        if timing:
            self.last_timing = {"op_to_host_s": time.perf_counter() - t0,
                                "kernel_ms": [a.elapsed_time(b) for a, b in t_ev],
                                "blocks_sent_at_mix": unsent, "blocks": self.nblk}
        self._done = None

    @property
    def pending(self):
        return self._done is not None

    def current(self):
        """The device outputs still hold the models' current values (see `fresh`)."""
        return self.fresh and (self.version_of is None or self.version_of() == self.models_version)


def mixing_op(dev, part, mixer):
    """ResidentRound device op of the plain round: Θ' = Wᵀ Θ with the stripe's Mixer (kept in
    part['mixer'], replaced on a new topology)."""
    part["mixer"] = mixer

    def op(ins, outs, mode, kernel):
        part["mixer"](ins[0], out=outs[0], mode=mode, kernel=kernel)
    return op


def fused_op(dev, part, grad_op, step_rows, lr, mixer, grad_writeback=True):
    """ResidentRound device op of the round with gradient averaging (FusedRoundRunner's per-window
    arithmetic on the whole stripe): ins = [params, grads] -> averaged gradients (outs[1]) -> SGD
    step of the stepped rows on the parameters in place -> mixing into outs[0].  grad_op None: the
    plain round's device step (each node's own gradient, d_sgd.py:51-52), no averaging."""
    from . import ops
    part["mixer"] = mixer
    rows = torch.as_tensor(step_rows, dtype=torch.int32).to(dev)
    neg_lr = -float(lr)

    def op(ins, outs, mode, kernel):
        xp, xg = ins
        if grad_op is None:
            gm = xg
        elif len(outs) > 1:
            gm = outs[1]
        else:                                 # no write-back of the averaged gradients
            if "dm" not in part:
                part["dm"] = torch.empty_like(xg)
            gm = part["dm"]
        if grad_op is not None:
            grad_op(xg, out=gm)
        if rows.numel():
            ops.sgd_step_rows(xp, gm, rows, neg_lr)
        part["mixer"](xp, out=outs[0], mode=mode, kernel=kernel)
    return op
