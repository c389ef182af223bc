"""Read guard for the deferred write-back of the row-streamed round.

niidmix.d_sgd.next_step may return while the mixed rows are still streaming back D2H into the
nodes' models (niidmix.slab.ResidentRound, deferred write-back): it predicts run.py's reads
(should_log, run.py:19-25; log_consensus_distance, run.py:118-119) and waits when the driver will
read.  Any OTHER reader between rounds -- a custom logger, a checkpoint, an evaluation hook -- would
otherwise see the pre-round parameters.  This module closes that gap: the models a resident engine
streams get a per-class subclass (cached, same name) whose Module entry points that read or write
parameters first wait for that model's own block of rows:

    forward / __call__, parameters, named_parameters, state_dict, load_state_dict, _apply (.to,
    .cuda, .float, ...)

A wait is one event synchronize of the model's row block (a no-op once the block is back), and it
is skipped entirely while no round is pending.  Reads through tensor references taken BEFORE the
round (a cached `list(model.parameters())`) bypass any Module method and are not covered:
call niidmix.d_sgd.synchronize() first.  NIIDMIX_READ_GUARD=0 disables the guard.
"""
import os
import weakref

# waits the guard performed (tests/test_gpu_dropin.py checks it fired)
stats = {"waits": 0}
_classes = {}
_suspend = [0]


def enabled():
    return os.environ.get("NIIDMIX_READ_GUARD", "1") != "0"


def _wait(model):
    if _suspend[0]:
        return
    tag = model.__dict__.get("_niidmix_row")
    if tag is None:
        return
    ref, i = tag[0], tag[1]
    eng = ref()
    if eng is not None and eng.pending:
        eng.wait_row(i)
        stats["waits"] += 1


def _stale(model):
    tag = model.__dict__.get("_niidmix_row")
    eng = tag[0]() if tag is not None else None
    if eng is not None:
        eng.fresh = False


def guarded_class(cls):
    """The guarded subclass of an nn.Module class (built once per class)."""
    if getattr(cls, "_niidmix_guarded", False):
        return cls
    g = _classes.get(cls)
    if g is not None:
        return g

    def forward(self, *a, **k):
        _wait(self)
        return cls.forward(self, *a, **k)

    def parameters(self, recurse=True):
        _wait(self)
        return cls.parameters(self, recurse)

    def named_parameters(self, *a, **k):
        _wait(self)
        return cls.named_parameters(self, *a, **k)

    def state_dict(self, *a, **k):
        _wait(self)
        return cls.state_dict(self, *a, **k)

    def load_state_dict(self, *a, **k):
        _wait(self)                    # a write: the pending D2H would overwrite it
        _stale(self)                   # and the resident device copy no longer matches
        return cls.load_state_dict(self, *a, **k)

    def _apply(self, *a, **k):
        _wait(self)
        _stale(self)
        return cls._apply(self, *a, **k)

    g = type(cls.__name__, (cls,), {
        "forward": forward, "parameters": parameters, "named_parameters": named_parameters,
        "state_dict": state_dict, "load_state_dict": load_state_dict, "_apply": _apply,
        "__module__": cls.__module__, "__qualname__": getattr(cls, "__qualname__", cls.__name__),
        "_niidmix_guarded": True})
    _classes[cls] = g
    return g


def first_param_ptr(model):
    with suspended():
        for q in model.parameters():
            return q.data_ptr()
    return None


def install(models, engine):
    """Tag `models` as rows of `engine` (row i = models[i]; engine: an object with .pending,
    .wait_row(i) and .fresh -- niidmix.slab.ResidentRound -- held weakly) and, unless
    NIIDMIX_READ_GUARD=0, guard them.  The tag also records where the model's first parameter
    lives (a slab view), so a deepcopy of the model -- which copies the tag -- is never taken for
    the row itself (resident_rows)."""
    ref = weakref.ref(engine)
    on = enabled()
    for i, m in enumerate(models):
        if on:
            m.__class__ = guarded_class(type(m))
        m.__dict__["_niidmix_row"] = (ref, i, first_param_ptr(m))


def resident_rows(models):
    """(engine, rows) when every model is a tagged, still slab-backed row of ONE engine, else
    None."""
    return _rows_of(models, "_niidmix_row")


def tag_slab(models, slab):
    """Record that models[i]'s parameters are row i of the pinned host slab `slab` (NodeSlab)."""
    ref = weakref.ref(slab)
    for i, m in enumerate(models):
        m.__dict__["_niidmix_slab"] = (ref, i, first_param_ptr(m))


def _rows_of(models, key):
    owner, rows = None, []
    for m in models:
        tag = m.__dict__.get(key)
        if tag is None:
            return None
        e = tag[0]()
        if e is None or (owner is not None and e is not owner) or first_param_ptr(m) != tag[2]:
            return None
        owner = e
        rows.append(tag[1])
    return (owner, rows) if owner is not None else None


def slab_rows(models):
    """(NodeSlab, rows) when every model is a still-backed row of ONE parameter slab, else None."""
    return _rows_of(models, "_niidmix_slab")


def strip(model):
    """Drop the row and slab tags of a copy (setup.model.average's deepcopy of models[0])."""
    model.__dict__.pop("_niidmix_row", None)
    model.__dict__.pop("_niidmix_slab", None)
    return model


class suspended:
    """Internal bookkeeping that only inspects parameter identities (NodeSlab.owns) while a round
    is pending: no wait."""

    def __enter__(self):
        _suspend[0] += 1

    def __exit__(self, *exc):
        _suspend[0] -= 1
