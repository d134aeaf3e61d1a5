"""Parameterized plan cache: queries that differ only in literal values share one planning.

Planning a query — optimizer batches, the Hyperspace rules (candidate indexes, signatures,
rankers), physical planning and ``EnsureRequirements`` — costs 0.2-0.5 ms of Python per query,
which is a large share of an indexed query that runs 0.3-1.5 ms on an MI355X.  A serving
workload repeats a handful of query *shapes* with new literals (TPC-H Q6 with another year,
Q3 with another date), and nothing in planning depends on literal values:

* the optimizer rules used here are structural, except ``OptimizeIn`` (it deduplicates IN-list
  values), so plans containing ``In``/``InSet`` are not parameterized;
* the Hyperspace rules decide from referenced columns, index metadata and file signatures;
* physical planning decides from sizes and partitioning, not from literals.

So the analyzed plan is fingerprinted with every literal replaced by a typed placeholder (its
type and null-ness stay in the key), attribute ids canonicalized by first appearance, and
relations by identity.  The key also carries the session state planning reads: the conf
version, the installed optimizer rules (Hyperspace enabled or not) and the identity of the
index-metadata snapshot the rules see (a refresh / create / delete or the TTL expiry of the
index cache produces a new snapshot, so a new key).

On a miss the query is planned normally and cached only if every literal object of the
analyzed plan survived, by identity, into the executed plan.  On a hit the cached executed plan
is copied with each old literal object replaced by the new query's literal in the same position.
Only the objects on paths from the plan root to those literals (recorded when the entry is
stored) are copied; everything else is shared with the cached plan.
"""
from __future__ import annotations

import copy
import threading
import weakref
from collections import OrderedDict
from typing import Dict, List, Optional, Tuple

import pyarrow as pa

from . import expressions as E
from . import logical as L

_PLAN_MODULES = ("hyperspace_amd.plan",)
_SCALARS = (str, int, float, bool, type(None), pa.DataType, pa.Schema, pa.Field)
CAPACITY = 256


class _NotCacheable(Exception):
    pass


class _Ctx:
    __slots__ = ("ids", "lits", "refs", "reuse")

    def __init__(self):
        self.ids: Dict[int, int] = {}
        self.lits: List[E.Literal] = []
        self.refs: list = []
        self.reuse = False   # a hit must run exchange reuse on the substituted plan

    def eid(self, x: int) -> int:
        v = self.ids.get(x)
        if v is None:
            v = len(self.ids)
            self.ids[x] = v
        return v


def _own(obj) -> bool:
    return type(obj).__module__.startswith(_PLAN_MODULES)


_PRIMS = (str, int, float, bool, type(None))
_SKIP = ("_cache", "_hs_")
_OWN: Dict[type, bool] = {}
_FIELDS: Dict[tuple, tuple] = {}


def _own_type(t: type) -> bool:
    o = _OWN.get(t)
    if o is None:
        o = _OWN[t] = t.__module__.startswith(_PLAN_MODULES) and not issubclass(t, L.HadoopFsRelation)
    return o


def _fields(d: dict) -> tuple:
    """Sorted fingerprinted field names of a node's ``__dict__`` (memoized by key set)."""
    ks = tuple(d)
    f = _FIELDS.get(ks)
    if f is None:
        # memoized derived state (_cache*, _hs_*) is not part of the node's meaning
        f = _FIELDS[ks] = tuple(sorted(k for k in ks if not k.startswith(_SKIP)))
    return f


def _fp_lit(v, ctx: _Ctx):
    ctx.lits.append(v)
    return ("L", str(v.dtype), v.value is None)


def _fp_attr(v, ctx: _Ctx):
    return ("A", v.name, str(v.dtype), v.nullable, ctx.eid(v.expr_id), v.qualifier)


def _fp_children(v, ctx: _Ctx):
    d = v.__dict__
    if len(d) != 1:                     # an instance with more fields: the generic walk
        return _fp_node(v, type(v), ctx)
    return (type(v).__name__, (("children", tuple([_fp(x, ctx) for x in d["children"]])),))


# per exact type: the fingerprint function the generic dispatch below would reach (the
# expression trees a serving loop builds per query are mostly these)
_FAST: Dict[type, object] = {}


def _fp(v, ctx: _Ctx):
    t = type(v)
    if t in _PRIMS:
        return v
    f = _FAST.get(t)
    if f is not None:
        return f(v, ctx)
    if t is tuple or t is list:
        return tuple([_fp(x, ctx) for x in v])
    if isinstance(v, E.Literal):
        _FAST[t] = _fp_lit
        return _fp_lit(v, ctx)
    if isinstance(v, (E.In, E.InSet)):
        raise _NotCacheable("IN list (OptimizeIn depends on its values)")
    if isinstance(v, E.Attribute):
        _FAST[t] = _fp_attr
        return _fp_attr(v, ctx)
    if isinstance(v, _PRIMS):
        return v
    if isinstance(v, (list, tuple)):
        return tuple(_fp(x, ctx) for x in v)
    if isinstance(v, (set, frozenset)):
        raise _NotCacheable("set-valued node field")
    if isinstance(v, dict):
        return tuple(sorted((str(k), _fp(x, ctx)) for k, x in v.items()))
    if isinstance(v, (pa.DataType, pa.Schema, pa.Field)):
        return str(v)
    if not _own_type(t):
        # relations, file indexes, tables: by identity (the entry keeps them alive)
        ctx.refs.append(v)
        return ("O", id(v))
    if t is L.LogicalRelation:
        return _fp_leaf(v, ctx)
    return _fp_node(v, t, ctx)


# A serving loop builds every query over the same base relation objects: their fingerprint is
# kept in local attribute numbering and re-mapped into the query's numbering on reuse.
_LEAF_FP: "weakref.WeakKeyDictionary" = weakref.WeakKeyDictionary()


def _fp_leaf(v, ctx: _Ctx):
    hit = _LEAF_FP.get(v)
    if hit is None:
        lctx = _Ctx()
        lfp = _fp_node(v, type(v), lctx)
        if lctx.lits:   # literals must reach the caller's list in order: no memo
            ctx.lits.extend(lctx.lits)
            ctx.refs.extend(lctx.refs)
            return ("LR", lfp, tuple(ctx.eid(x) for x in lctx.ids))
        hit = _LEAF_FP[v] = (lfp, tuple(lctx.ids), tuple(lctx.refs))
    lfp, ids, refs = hit
    ctx.refs.extend(refs)
    return ("LR", lfp, tuple([ctx.eid(x) for x in ids]))


def _fp_node(v, t: type, ctx: _Ctx):
    d = vars(v)
    fields = _fields(d)
    if fields == ("children",) and type(d["children"]) is tuple and t not in _FAST:
        _FAST[t] = _fp_children        # its fingerprint is its type and its children's
    items = []
    for k in fields:
        x = d[k]
        items.append((k, ctx.eid(x)) if k == "expr_id" else (k, _fp(x, ctx)))
    return (t.__name__, tuple(items))


# Native walk (csrc/host/hs_host.cpp, same output as ``_fp``): per exact type a (code, name)
# pair - 0 generic node, 1 literal, 2 attribute, 3 children-only node, 4 the Python ``_fp``
_KINDS: Dict[type, tuple] = {}


def _classify(t: type) -> tuple:
    if issubclass(t, E.Literal):
        k = 1
    elif issubclass(t, (E.In, E.InSet)):
        k = 4
    elif issubclass(t, E.Attribute):
        k = 2
    elif t is L.LogicalRelation:
        k = 5
    elif issubclass(t, _PRIMS + (list, tuple, set, frozenset, dict, pa.DataType, pa.Schema,
                                 pa.Field)) or not _own_type(t):
        k = 4
    else:
        k = 3
    out = _KINDS[t] = (k, t.__name__)
    return out


_HOST_ABI = 2      # csrc/host/hs_host.cpp ``ABI``


def _native():
    try:
        import importlib.util
        from .._native.build import host_ext_path
        path = host_ext_path()
        spec = importlib.util.spec_from_file_location("_hs_host", path)
        if spec is None or not __import__("os").path.exists(path):
            return None
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        return mod if getattr(mod, "ABI", None) == _HOST_ABI else None
    except (ImportError, OSError):
        return None


_NATIVE = _native()
_NATIVE_FP = _NATIVE.fingerprint if _NATIVE is not None else None


def _leaf_memo(v):
    """(fingerprint in local numbering, expr ids, refs) of base relation ``v`` (``_fp_leaf``'s
    memo), or None when it holds literals (no memo: the Python walk handles it)."""
    hit = _LEAF_FP.get(v)
    if hit is None:
        lctx = _Ctx()
        lfp = _fp_node(v, type(v), lctx)
        if lctx.lits:
            return None
        hit = _LEAF_FP[v] = (lfp, tuple(lctx.ids), tuple(lctx.refs))
    return hit


def fingerprint(logical, ctx: _Ctx, native: Optional[bool] = None):
    """The plan-cache fingerprint of ``logical`` (``_fp``), through the native walk when it is
    built (``native`` None) or as asked."""
    f = _NATIVE_FP if native is not False else None
    if native and f is None:
        raise RuntimeError("_hs_host extension not built")
    if f is None:
        return _fp(logical, ctx)
    return f(logical, ctx.ids, ctx.lits, ctx.refs, _KINDS, _classify, _fields,
             lambda v: _fp(v, ctx), _leaf_memo)


def _iter_literals(v, out: List[E.Literal], seen: set):
    """Every Literal object reachable from a plan (through our own node/container types)."""
    if isinstance(v, E.Literal):
        out.append(v)
        return
    if isinstance(v, _SCALARS):
        return
    if isinstance(v, (list, tuple, set, frozenset)):
        for x in v:
            _iter_literals(x, out, seen)
        return
    if isinstance(v, dict):
        for x in v.values():
            _iter_literals(x, out, seen)
        return
    if not _own(v) or isinstance(v, L.HadoopFsRelation) or id(v) in seen:
        return
    seen.add(id(v))
    for x in vars(v).values():
        _iter_literals(x, out, seen)


def _hot_paths(v, lit_ids: set, hot: set, seen: Dict[int, bool]) -> bool:
    """Mark (in ``hot``) every object/container on a path from ``v`` to a literal in
    ``lit_ids``; returns whether ``v`` leads to one."""
    if isinstance(v, E.Literal):
        return id(v) in lit_ids
    if isinstance(v, _SCALARS):
        return False
    k = id(v)
    if k in seen:
        return seen[k]
    seen[k] = False
    found = False
    if isinstance(v, (list, tuple)):
        for x in v:
            found = _hot_paths(x, lit_ids, hot, seen) or found
    elif isinstance(v, dict):
        for x in v.values():
            found = _hot_paths(x, lit_ids, hot, seen) or found
    elif _own(v) and not isinstance(v, (L.HadoopFsRelation, L.LogicalPlan)):
        for x in vars(v).values():
            found = _hot_paths(x, lit_ids, hot, seen) or found
    seen[k] = found
    if found:
        hot.add(k)
    return found


def _subst(v, m: Dict[int, E.Literal], hot: set, memo: Dict[int, object]):
    """Copy of ``v`` with literal objects replaced via ``m`` (id -> new literal), rebuilding only
    the objects on ``hot`` paths; everything else is shared with the cached plan."""
    if isinstance(v, E.Literal):
        return m.get(id(v), v)
    k = id(v)
    if k not in hot:
        return v
    hit = memo.get(k)
    if hit is not None:
        return hit
    if isinstance(v, list):
        out = [_subst(x, m, hot, memo) for x in v]
    elif isinstance(v, tuple):
        out = tuple(_subst(x, m, hot, memo) for x in v)
    elif isinstance(v, dict):
        out = {kk: _subst(x, m, hot, memo) for kk, x in v.items()}
    else:
        d = vars(v)
        if type(v).__reduce_ex__ is object.__reduce_ex__ and not hasattr(v, "__slots__"):
            # plain node: shallow copy without copy.copy's reduce protocol (hot on cache hits)
            out = object.__new__(type(v))
            nd = out.__dict__
            nd.update(d)
            for kk, x in d.items():
                nx = _subst(x, m, hot, memo)
                if nx is not x:
                    nd[kk] = nx
        else:
            out = copy.copy(v)
            for kk, x in d.items():
                nx = _subst(x, m, hot, memo)
                if nx is not x:
                    object.__setattr__(out, kk, nx)
    memo[k] = out
    return out


def _deferred_literals(plan) -> set:
    """ids of the literals a backend evaluates after a query's submission returns: those in an
    aggregate's result expressions outside the aggregate functions' own inputs (the result
    arithmetic over aggregates runs when the result is fetched) and those in a global sort's
    order expressions (GpuBackend orders the few result rows on the host when the result is
    fetched, exec/gpu.py ``_collect_native``)."""
    from . import physical as X
    out: set = set()

    def walk(e):
        if isinstance(e, E.AggregateFunction):
            return
        if isinstance(e, E.Literal):
            out.add(id(e))
            return
        for c in getattr(e, "children", ()):
            walk(c)
    for n in plan.collect(lambda x: isinstance(x, X.HashAggregateExec)):
        for e in n.aggregates:
            walk(e)
    for n in plan.collect(lambda x: isinstance(x, X.SortExec) and x.global_sort):
        for o in n.order:
            walk(o.child)
    return out


class _Entry:
    """One cached executed plan.  Its literal objects are private clones (``old_lits``), so a
    hit can also run the cached plan itself with the new query's values written into them for
    the duration of a submission (``bind_literals`` / ``restore_literals`` under ``lock``): no
    plan copy, and the executor sees the same node objects on every hit (its per-node memos
    stay warm).  ``inplace_ok`` is False when a literal sits where a submitted query still
    reads it after the submission returns (a result expression over aggregates, evaluated when
    the result is fetched); such entries are always materialized."""
    __slots__ = ("plan", "old_lits", "paths", "refs", "reuse", "lock", "inplace_ok")

    def __init__(self, plan, old_lits, paths, refs, reuse, inplace_ok=False):
        self.plan, self.old_lits, self.paths, self.refs, self.reuse = \
            plan, old_lits, paths, refs, reuse
        self.lock = threading.Lock()
        self.inplace_ok = inplace_ok

    def bind_literals(self, lits) -> list:
        """Write the new query's literal values into the cached plan's literal objects (caller
        holds ``lock``); returns what ``restore_literals`` puts back."""
        saved = []
        for o, n in zip(self.old_lits, lits):
            if o is not n:
                saved.append((o, o.value))
                o.value = n.value
        return saved

    @staticmethod
    def restore_literals(saved) -> None:
        for o, v in saved:
            o.value = v


class PlanCache:
    def __init__(self, capacity: int = CAPACITY):
        self.capacity = capacity
        self._lru: "OrderedDict[tuple, tuple]" = OrderedDict()
        self._lock = threading.Lock()
        self.hits = 0
        self.misses = 0
        self.uncacheable = 0

    @staticmethod
    def _session_key(session, ctx: _Ctx) -> tuple:
        rules = tuple(id(r) for r in session.extra_optimizations)
        ctx.refs.extend(session.extra_optimizations)
        snap = 0
        if session.extra_optimizations:
            from ..hyperspace import get_context
            snap_obj = get_context(session).index_collection_manager.snapshot()
            ctx.refs.append(snap_obj)
            snap = id(snap_obj)
        return (id(session), session.conf.version, rules, snap)

    def lookup_entry(self, session, logical):
        """(entry or None, key, fingerprint context) of ``logical`` - no substitution.  A hit's
        ``ctx.lits`` are the new query's literals, position for position with
        ``entry.old_lits``."""
        ctx = _Ctx()
        try:
            key = (self._session_key(session, ctx), fingerprint(logical, ctx))
        except _NotCacheable:
            self.uncacheable += 1
            return None, None, ctx
        with self._lock:
            hit = self._lru.get(key)
            if hit is not None:
                self._lru.move_to_end(key)
        if hit is None or len(hit.old_lits) != len(ctx.lits):
            self.misses += 1
            return None, key, ctx
        ctx.reuse = hit.reuse
        self.hits += 1
        return hit, key, ctx

    def materialize(self, entry: "_Entry", ctx: _Ctx):
        """The cached executed plan with the new query's literals (``ctx.lits``) substituted
        along their paths.  Every literal position is replaced, changed value or not: the
        entry's own literal objects are rewritten in place by concurrent bound submissions
        (``_Entry.bind_literals``), so no materialized plan may share them.  Runs
        under ``entry.lock`` so the entry's paths and literal list are read consistently."""
        with entry.lock:
            m = {}
            for o, n in zip(entry.old_lits, ctx.lits):
                m[id(o)] = n if n is not o else copy.copy(n)
            if not m:
                return entry.plan
            hot = set().union(*(entry.paths[k] for k in m))
            return _subst(entry.plan, m, hot, {})

    def lookup(self, session, logical) -> Tuple[Optional[object], Optional[tuple], _Ctx]:
        """(executed plan or None, key, fingerprint context) of ``logical``."""
        entry, key, ctx = self.lookup_entry(session, logical)
        if entry is None:
            return None, key, ctx
        return self.materialize(entry, ctx), key, ctx

    def store(self, key, executed, ctx: _Ctx):
        """Cache ``executed`` — the plan *before* exchange reuse — for ``key`` if every literal
        of the analyzed plan reached it.  Exchange reuse compares canonical subtrees including
        literal values (a self-join with equal filter literals shares one exchange, with unequal
        ones it must not), so it is never part of a cached plan: entries whose plan has two
        exchanges that could match are flagged and re-run ``reuse_exchanges`` after each
        substitution."""
        if key is None:
            return None
        from . import physical as X
        exch = executed.collect(lambda n: isinstance(n, (X.ShuffleExchangeExec,
                                                         X.BroadcastExchangeExec)))
        shapes = [(type(e).__name__, len(e.output), type(getattr(e, "partitioning", None)).__name__,
                   getattr(getattr(e, "partitioning", None), "num_partitions", None))
                  for e in exch]
        reuse = len(shapes) != len(set(shapes))
        if reuse:
            # two exchanges can only ever be reused when they read the same data: exchanges of
            # one shape over different scans (a Hybrid Scan join's two appended-file shuffles)
            # never match, whatever the literals - no reuse pass per hit for them
            def data_id(e):
                return tuple(sorted(
                    (type(n.relation.location).__name__,
                     hash(tuple(sorted(repr(f) for f in n.relation.location.all_files()))))
                    if isinstance(n, X.FileSourceScanExec) else
                    (("local", id(n.table)) if isinstance(n, X.LocalTableScanExec)
                     else (type(n).__name__,))
                    for n in e.collect(lambda m: not m.children)))
            keyed = [(sh, data_id(e)) for sh, e in zip(shapes, exch)]
            reuse = len(keyed) != len(set(keyed))
        present: List[E.Literal] = []
        _iter_literals(executed, present, set())
        ids = {id(x) for x in present}
        if not all(id(x) in ids for x in ctx.lits):
            self.uncacheable += 1
            return None
        paths = {}
        for x in ctx.lits:
            if id(x) not in paths:
                hot: set = set()
                _hot_paths(executed, {id(x)}, hot, {})
                paths[id(x)] = hot
        # the entry's own copy, with private literal objects: the caller keeps running (and may
        # re-execute) ``executed``, whose literals must never see another query's values
        clones = {k: copy.copy(x) for k, x in ((id(x), x) for x in ctx.lits)}
        private = _subst(executed, clones, set().union(*paths.values()) if paths else set(), {})
        old_lits = [clones[id(x)] for x in ctx.lits]
        ppaths = {}
        for x in old_lits:
            if id(x) not in ppaths:
                hot = set()
                _hot_paths(private, {id(x)}, hot, {})
                ppaths[id(x)] = hot
        late = _deferred_literals(private)
        entry = _Entry(private, old_lits, ppaths, list(ctx.refs), reuse,
                       inplace_ok=not any(id(x) in late for x in old_lits))
        with self._lock:
            self._lru[key] = entry
            while len(self._lru) > self.capacity:
                self._lru.popitem(last=False)
        return entry

    def clear(self):
        with self._lock:
            self._lru.clear()


def plan_cache(session) -> PlanCache:
    pc = getattr(session, "_plan_cache", None)
    if pc is None:
        pc = PlanCache()
        session._plan_cache = pc
    return pc
