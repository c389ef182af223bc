"""Read guard for the deferred write-back of the row-streamed round.

niidmix.d_sgd.next_step may return while the mixed rows are still streaming back D2H into the
nodes' models (niidmix.slab.ResidentRound, deferred write-back): it predicts run.py's reads
(should_log, run.py:19-25; log_consensus_distance, run.py:118-119) and waits when the driver will
read.  Any OTHER reader between rounds -- a custom logger, a checkpoint, an evaluation hook -- would
otherwise see the pre-round parameters.  This module closes that gap: the models a resident engine
streams get a per-class subclass (cached, same name) whose Module entry points that read or write
parameters first wait for that model's own block of rows:

    forward / __call__, parameters, named_parameters, state_dict, load_state_dict, _apply (.to,
    .cuda, .float, ...), and pickling / deepcopy (__reduce_ex__)

A wait is one event synchronize of the model's row block (a no-op once the block is back), and it
is skipped entirely while no round is pending.  Reads through tensor references taken BEFORE the
round (a cached `list(model.parameters())`) bypass any Module method and are not covered:
call niidmix.d_sgd.synchronize() first.  NIIDMIX_READ_GUARD=0 disables the guard.

Pickling.  A guarded model pickles (torch.save, pickle, a torch.multiprocessing queue, deepcopy)
as an instance of its ORIGINAL class: __reduce_ex__ waits for the row, then names the base class,
so the unpickled model is a plain model holding the mixed values.  The row / slab tags live in
module-level weak dictionaries keyed by the model, never in the model's __dict__, so no weakref or
engine reference travels with a pickled or copied model (a copy is never taken for the row).
"""
import copyreg
import os
import weakref

# waits the guard performed (tests/test_gpu_dropin.py checks it fired)
stats = {"waits": 0}
_classes = {}
_suspend = [0]
# model -> (weakref to the owning ResidentRound, row, first parameter's data_ptr)
_row_tags = weakref.WeakKeyDictionary()
# model -> (weakref to the owning NodeSlab, row, first parameter's data_ptr)
_slab_tags = weakref.WeakKeyDictionary()


def enabled():
    return os.environ.get("NIIDMIX_READ_GUARD", "1") != "0"


def row_tag(model):
    """The (engine ref, row, first parameter pointer) tag install() gave `model`, or None."""
    return _row_tags.get(model)


def _wait(model):
    if _suspend[0]:
        return
    tag = _row_tags.get(model)
    if tag is None:
        return
    ref, i = tag[0], tag[1]
    eng = ref()
    if eng is not None and eng.pending:
        eng.wait_row(i)
        stats["waits"] += 1


def _stale(model):
    tag = _row_tags.get(model)
    eng = tag[0]() if tag is not None else None
    if eng is not None:
        eng.fresh = False


def _as_base(obj, g, cls):
    if obj is g:
        return cls
    if isinstance(obj, tuple):
        return tuple(_as_base(o, g, cls) for o in obj)
    return obj


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

    def __reduce_ex__(self, protocol):
        # pickle / torch.save / deepcopy read the parameters: wait for the row, then reduce as
        # the base class (the guarded class is not importable under its name)
        _wait(self)
        rv = super(g, self).__reduce_ex__(protocol)
        if not isinstance(rv, tuple) or len(rv) < 2:
            return rv
        if rv[0] is copyreg.__newobj__ and rv[1] == (g,):
            # the pickler insists that __newobj__'s class is the object's own: rebuild through
            # the stdlib's object.__new__(cls) instead (no niidmix import needed to unpickle)
            return (copyreg._reconstructor, (cls, object, None)) + rv[2:]
        return (rv[0], _as_base(rv[1], g, cls)) + rv[2:]

    g = type(cls.__name__, (cls,), {
        "forward": forward, "parameters": parameters, "named_parameters": named_parameters,
        "state_dict": state_dict, "load_state_dict": load_state_dict, "_apply": _apply,
        "__reduce_ex__": __reduce_ex__,
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
    lives (a slab view), so a model whose parameters were re-pointed elsewhere is no longer taken
    for the row (resident_rows)."""
    ref = weakref.ref(engine)
    on = enabled()
    for i, m in enumerate(models):
        if on:
            m.__class__ = guarded_class(type(m))
        _row_tags[m] = (ref, i, first_param_ptr(m))


def resident_rows(models):
    """(engine, rows) when every model is a tagged, still slab-backed row of ONE engine, else
    None."""
    return _rows_of(models, _row_tags)


def tag_slab(models, slab):
    """Record that models[i]'s parameters are row i of the pinned host slab `slab` (NodeSlab)."""
    ref = weakref.ref(slab)
    for i, m in enumerate(models):
        _slab_tags[m] = (ref, i, first_param_ptr(m))


def _rows_of(models, tags):
    owner, rows = None, []
    for m in models:
        tag = tags.get(m)
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
    return _rows_of(models, _slab_tags)


def strip(model):
    """Drop any row / slab tag of `model` (setup.model.average's deepcopy of models[0]: tags are
    never copied, so this only guards against a caller handing back a tagged model itself)."""
    _row_tags.pop(model, None)
    _slab_tags.pop(model, None)
    return model


class suspended:
    """Internal bookkeeping that only inspects parameter identities (NodeSlab.owns) while a round
    is pending: no wait."""

    def __enter__(self):
        _suspend[0] += 1

    def __exit__(self, *exc):
        _suspend[0] -= 1
