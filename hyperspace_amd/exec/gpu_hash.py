"""Hash-mode GROUP BY: device hash tables over scans and the run-keyed merge join, functional-
dependency grouping, the run top-K for ORDER BY <aggregate> LIMIT k, device top-k candidates
and the cross-rank merge."""
from __future__ import annotations

from typing import Optional

import numpy as np
import pyarrow as pa

from ..ops import _lib as NL, kernels as K
from ..plan import expressions as E, physical as X
from ..utils import murmur3
from ..utils.conf import HyperspaceConf
from ..utils.tracing import stage
from . import compile as CP, jit
from .arrow_eval import key
from .gpu_common import (arrow_table, _HashPrep, _eval_vec, _fd_columns, _finalize_array,
                         _gather_tables, DRel, H_TOPK_K, TOPK_MIN_GROUPS, Unsupported)


class HashAggOps:
    """Hash aggregate operators of ``GpuBackend`` (exec/gpu.py)."""

    # ------------------------------------------------------------------------------------------
    # Hash-mode aggregation (multi-column / high-cardinality / float keys; exec/hash_agg.py)
    # ------------------------------------------------------------------------------------------
    def _hash_agg(self, final: X.HashAggregateExec, child: X.SparkPlan, order, limit):
        """GROUP BY through the device hash table: every (part) launch of the fused scan or
        merge-join kernel inserts into one table, ``hs_hagg_extract`` compacts it, ranks merge
        their groups, and ORDER BY ... LIMIT picks its candidates on the device.  Kernels and the
        extract are queued now; ``finish`` reads the group count (re-running with a 4x table if
        the size guess overflowed) and copies the result."""
        from . import hash_agg as H
        if not HyperspaceConf.codegen_enabled(self.session.conf):
            raise Unsupported("hash aggregate needs code generation")
        fns = [fn for _, fn in X.agg_functions(final.aggregates)]
        grouping = list(final.grouping)
        if not all(isinstance(g, E.Attribute) for g in grouping):
            raise Unsupported("group by expression")
        node = child
        while isinstance(node, X.ProjectExec) and \
                all(isinstance(e, E.Attribute) for e in node.project_list):
            node = node.child
        # a plan-cache hit re-submits the same plan nodes with new literals: the relations,
        # grouping, domains and top-K request are kept per aggregate node (``_HashPrep``), and
        # the lowering of each literal vector (join parameters, key plan, ranges) with them
        prep = self._hash_prep_get(final, order, limit)
        if prep is not None:
            (left, right, lk, rk, rels, launches, fd, grouping, doms, A, minmax, shape_key, est,
             tk_req) = prep.setup
        else:
            fd = None
            left = right = lk = rk = None
            if isinstance(node, X.SortMergeJoinExec) and node.join_type == "inner":
                left, right, lk, rk = self._join_inputs(node)
                lparts, rparts = left.parts or [left], right.parts or [right]
                rels = lparts + rparts
                launches = [("join", lp, rp) for lp in lparts for rp in rparts]
                fd = self._fd_grouping(final, grouping, left, right, lk, rk, order, limit)
                if fd is not None:
                    grouping = fd[0]
            else:
                r = self._rel(child)
                rels = r.parts or [r]
                launches = [("scan", x, None) for x in rels]
            doms = {g.expr_id: self._union_domain(rels, g) for g in grouping}
            A = len(fns) + 1
            minmax = any(isinstance(fn, (E.Min, E.Max)) for fn in fns)
            shape_key = (tuple(g.name for g in grouping), tuple(fn.sql() for fn in fns),
                         tuple(id(x.table) for x in rels))
            est = min(sum(x.table.num_rows or 0 for x in rels), 1 << 40)
            span = 1
            for g in grouping:
                span *= max(1, doms[g.expr_id][1]) + 1 if doms[g.expr_id][1] else (1 << 32)
            est = max(1, min(est, span))
            # ORDER BY <sum / count> LIMIT k over the key-run hash walk: whole keys compete in
            # the walk's per-wavefront top-K lists and only split keys use the table (TopKPlan)
            tk_req = self._topk_request(final, fns, order, limit, minmax) \
                if fd is not None else None
            prep = self._hash_prep_put(final, order, limit, node, launches, (
                left, right, lk, rk, rels, launches, fd, grouping, doms, A, minmax, shape_key,
                est, tk_req))
        hk_box: list = []
        tk_box: list = []

        def run(M: int, use_tk: bool = True):
            table = self.htables.get(M, A, minmax, self.device)
            tk_box.clear()
            with stage("hagg.kernels"):
                for kind, a, b in launches:
                    if kind == "join":
                        self._join_hash_pair(node, a, b, lk, rk, fns, grouping, doms, table, hk_box,
                                             tk_req=tk_req if use_tk else None, tk_box=tk_box,
                                             prep=prep)
                    else:
                        self._scan_hash(a, fns, grouping, doms, table, hk_box)
            with stage("hagg.extract"):
                return table.extract(A - 1)

        M = self.htables.slots_for(shape_key, est)
        groups = run(M)
        d = self._dist()

        def finish() -> pa.Table:
            if fd is not None and d is not None and d.world > 1:
                # keys partitioned by bucket: this rank's top candidates, then result rows
                # from every rank (one exchange; the caller sorts and cuts)
                t = local()
                with stage("hagg.gather_rows"):
                    return _gather_tables(d, t)
            return local()

        def local() -> pa.Table:
            nonlocal groups, M
            with stage("hagg.result"):
                hk = hk_box[0] if hk_box else None
                tk = tk_box[0] if tk_box and tk_box[0].used else None
                if tk is not None and hk is not None:
                    # run top-K: candidates, the table's size and the candidates' right
                    # columns in one copy (_topk_fast, _fd_device)
                    fdd = self._fd_device(hk, right, rk, fd) if fd is not None else None
                    st, host, G = self._topk_fast(tk, groups, hk, A, int(limit), fdd)
                    while st == "over":
                        if M >= H.MAX_SLOTS:
                            raise Unsupported("hash aggregate table too large")
                        M *= 4
                        groups = run(M)
                        st, host, G = self._topk_fast(tk_box[0], groups, hk, A, int(limit), fdd)
                    self.htables.record(shape_key, M, G)
                    if st == "ok":
                        self.metrics["run_topk"] = 1
                        ex = None
                        if fd is not None and "fd" in host:
                            def ex(gmap, host):
                                _fd_columns(fd[1], fdd["cols"], host["fd"], gmap)
                        elif fd is not None:
                            def ex(gmap, host):
                                self._fd_lookup(right, rk, fd[1], gmap[fd[0][0].expr_id], gmap)
                        return self._hash_table_out(final, fns, grouping, hk, host, A, ex)
                    # a dropped value may tie the k-th one (or ties flood the copy): exact path
                    self.metrics["run_topk"] = 0
                    groups = run(M, use_tk=False)
                G, over = groups.count()
                while over:
                    if M >= H.MAX_SLOTS:
                        raise Unsupported("hash aggregate table too large")
                    M *= 4
                    groups = run(M, use_tk=False)
                    G, over = groups.count()
                self.htables.record(shape_key, M, G)
                extra = None
                if fd is not None:
                    def extra(gmap, host):
                        self._fd_lookup(right, rk, fd[1], gmap[fd[0][0].expr_id], gmap)
                if d is not None and d.world > 1 and fd is None:
                    groups, G = self._hash_combine_ranks(d, groups, G, A, minmax)
                if hk is None or G == 0:
                    return self._hash_table_out(final, fns, grouping, hk, None, A)
                src = self._topk_source(final, fns, grouping, hk, order, limit, G)
                if src is not None:
                    groups, G = H.topk_candidates(groups, G, src, int(limit))
                return self._hash_table_out(final, fns, grouping, hk, groups.to_host(G), A,
                                            extra)
        return finish

    # keys per functional-dependency lookup (one probe per key, in the key's bucket)
    FD_MAX_KEYS = 1 << 22

    def _fd_grouping(self, final, grouping, left: DRel, right: DRel, lk, rk, order, limit):
        """GROUP BY (left join key, right columns...) over an inner join whose right key is
        unique: every right column is a function of the key (TPC-H Q3's ``l_orderkey,
        o_orderdate, o_shippriority``), so the groups are the left key's and the right columns
        are looked up for the result groups only (``_fd_lookup``).  The reduced grouping lets
        the run-keyed two-phase join aggregate into the hash table (jit_runs hash walk).  Returns
        ([the key attribute], [right attributes]) or None.  Applies when the result is bounded
        by an ORDER BY <aggregate> LIMIT k (device top-k).  Sharded across ranks the key is
        both sides' bucket key, so every key's groups live on one rank: each rank finishes its
        own top candidates and the ranks exchange result rows only (``_gather_tables``); the
        table-dependent checks are agreed once per table pair, so every rank takes the same
        path."""
        if not HyperspaceConf.fd_group_enabled(self.session.conf):
            return None
        if left.parts or right.parts or not order or limit is None or \
                not 0 < int(limit) <= 1024:
            return None
        d = self._dist()
        if d is not None and d.world > 1:
            gk = (getattr(left.table, "global_key", None), getattr(right.table, "global_key", None),
                  lk.name, rk.name, tuple(g.name for g in grouping))
            if gk[0] is None or gk[1] is None:
                return None
            memo = self.__dict__.setdefault("_fd_agreed", {})
            ok = memo.get(gk)
            if ok is None:
                local = self._fd_grouping_local(final, grouping, left, right, lk, rk, order)
                ok = not d.agree_any([local is None])[0]
                memo[gk] = ok
            return self._fd_grouping_local(final, grouping, left, right, lk, rk, order,
                                           check=False) if ok else None
        return self._fd_grouping_local(final, grouping, left, right, lk, rk, order)

    def _fd_grouping_local(self, final, grouping, left: DRel, right: DRel, lk, rk, order,
                           check: bool = True):
        """``_fd_grouping`` on this rank's tables (``check``: the data-dependent checks too)."""
        if check and (right.table.num_rows or 0) * 64 < (left.table.num_rows or 0):
            return None          # _join_hash_pair would swap the sides
        keyg = [g for g in grouping if g.expr_id in (lk.expr_id, rk.expr_id)]
        rest = [g for g in grouping if g.expr_id not in (lk.expr_id, rk.expr_id)]
        if len(keyg) != 1 or not rest:
            return None
        if any(g.expr_id not in right.colmap or g.expr_id in left.colmap for g in rest):
            return None
        lc, rc = left.col(lk), right.col(rk)
        if lc.is_float or rc.is_float or lc.dictionary is not None or \
                rc.dictionary is not None or lc.valid is not None or \
                rc.hs_type not in (NL.I8, NL.I16, NL.I32, NL.I64):
            return None
        e = order[0].child
        if not isinstance(e, E.Attribute):
            return None
        ok = False
        for agg in final.aggregates:
            a = agg if isinstance(agg, E.Attribute) else agg.to_attribute()
            if a.expr_id == e.expr_id:
                inner = agg.child if isinstance(agg, E.Alias) else agg
                ok = isinstance(inner, E.AggregateFunction)
        if not ok or (check and jit.key_has_dups(rc)):
            return None
        g = keyg[0]
        if g.expr_id != lk.expr_id:      # the right key's attribute: group by the left's
            g = lk
        return [g], rest

    def _fd_lookup(self, right: DRel, rk, attrs, keys: pa.Array, gmap: dict) -> None:
        """``gmap[attr] = right[attr]`` at the right row of each key (unique right keys; the
        row is found by one equality probe in the key's bucket, as ``_probe_ranges``)."""
        import torch
        G = len(keys)
        if G == 0:
            for a in attrs:
                gmap[a.expr_id] = pa.array([], type=a.data_type)
            return
        if G > self.FD_MAX_KEYS:
            raise RuntimeError(f"functional-dependency lookup of {G} keys")
        rc = right.col(rk)
        width = {NL.I8: 8, NL.I16: 16, NL.I32: 32, NL.I64: 64}[rc.hs_type]
        vals = np.asarray(keys.cast(pa.int64()).to_numpy(zero_copy_only=False), dtype=np.int64)
        if width == 64:
            img = vals.view(np.uint64) ^ np.uint64(1 << 63)
        else:
            img = (vals + (1 << (width - 1))).astype(np.uint64)
        nb = len(right.table.bucket_offsets_host) - 1
        # each key probes only its own bucket (the index's Murmur3 bucketing of the right key)
        bids = np.asarray(murmur3.bucket_ids([keys.cast(rk.data_type)], nb), dtype=np.int32)
        # one upload (bucket ids and key images), rows picked on the device, one check after
        # the gathers are queued: the lookup synchronizes once before its column copies
        both = torch.from_numpy(np.concatenate([bids.astype(np.int64), img.view(np.int64)]))
        both = both.to(self.device)
        pb, pk = both[:G].to(torch.int32), both[G:]
        rstart, rlen, _ = K.probe_ranges(rc, right.table.bucket_offsets, pb, pk)
        idx = torch.where(rlen > 0, rstart, torch.zeros_like(rstart))
        cols = K.gather_columns([right.col(a) for a in attrs], idx)
        if int((rlen <= 0).sum().item()):
            raise RuntimeError("functional-dependency lookup: a group key has no right row")
        for a, c in zip(attrs, cols):
            arr = c.to_arrow()
            if not arr.type.equals(a.data_type):
                try:
                    arr = arr.cast(a.data_type)
                except (pa.ArrowInvalid, pa.ArrowNotImplementedError):
                    pass
            gmap[a.expr_id] = arr

    def _union_domain(self, rels, g: E.Attribute):
        """(lo, span, scale) of group column ``g`` over every part holding it and every rank.
        Integer columns: their value range (scale None).  float64 columns: the range of the
        exact decimal integers q = x * scale of their compact encoding (exec/encoding.py), so
        such a column packs into a multi-column key; scale 0.0 = no usable encoding (a float
        key then only runs alone, as raw bits).  Dictionary columns need none."""
        from .encoding import compact_of
        lo, hi, seen = None, None, False
        dicts = []
        scale = None
        for x in rels:
            if g.expr_id not in x.colmap:
                continue
            c = x.col(g)
            if c.dictionary is not None:
                dicts.append(c.dictionary)
                continue
            if c.is_float:
                enc = compact_of(c) if c.hs_type == NL.F64 else None
                if enc is None or enc.scale is None or enc.lo is None or \
                        (scale is not None and enc.scale != scale):
                    return (0, 0, 0.0)
                scale = enc.scale
                seen = True
                l0, sp = int(enc.lo), int(enc.hi) - int(enc.lo) + 1
            else:
                seen = True
                l0, sp = self._local_domain(c)
            if sp == 0:
                continue
            lo = l0 if lo is None else min(lo, l0)
            hi = l0 + sp - 1 if hi is None else max(hi, l0 + sp - 1)
        if len(dicts) > 1 and not all(dd.equals(dicts[0]) for dd in dicts[1:]):
            raise Unsupported("string group key with different dictionaries per part")
        d = self._dist()
        if seen and d is not None and d.world > 1:
            import torch
            dev = d.device if d.backend == "nccl" else "cpu"
            big = 1 << 62
            t = torch.tensor([-(lo if lo is not None else big), hi if hi is not None else -big],
                             dtype=torch.int64, device=dev)
            d.all_reduce(t, "max")
            nlo, nhi = -int(t[0].item()), int(t[1].item())
            if nhi < nlo:
                return (0, 0, scale)
            return (nlo, nhi - nlo + 1, scale)
        if lo is None:
            return (0, 0, scale)
        return (lo, hi - lo + 1, scale)

    def _hash_keyplan(self, grouping, col_info, fns, doms, specs, descs):
        from . import hash_agg as H
        items = []
        for g in grouping:
            ci = col_info(g)
            items.append((ci.slot, g, descs[ci.slot], doms[g.expr_id]))
        own = []
        for a in specs:
            own.append(a.kind != NL.AK_COUNT_STAR and
                       any(descs[a.col[t]].valid is not None for t in range(a.nterms)))
        need_star = any(isinstance(fn, (E.Count, E.Avg)) for fn in fns)
        return H.plan_keys(items, tuple(own), need_star)

    def _scan_hash(self, r: DRel, fns, grouping, doms, table, hk_box) -> None:
        col_info, descs = self._column_infos([(r, 0)])
        implied: set = set()
        spec = self._range_spec(r, r.conds, implied)
        with stage("scan.ranges"):
            rstart, rlen, _ = self._ranges(r, r.conds) if spec is not None else \
                self._full_ranges(r.table)
        bound = CP.bind(CP.to_cnf([c for c in r.conds if id(c) not in implied]), col_info,
                        self.device)
        specs = self._agg_specs(fns, col_info)
        hk = self._hash_keyplan(grouping, col_info, fns, doms, specs, descs)
        if not hk_box:
            hk_box.append(hk)
        p = NL.ScanParams()
        p.group_col, p.num_groups, p.group_base = -1, 1, 0
        for s, c in descs.items():
            p.cols[s] = c.desc()
        for i, pr in enumerate(bound.preds):
            p.preds[i] = pr
        p.npreds = len(bound.preds)
        for i, a in enumerate(specs):
            p.aggs[i] = a
        p.naggs = len(specs)
        if bound.always_false or (r.table.num_rows or 0) == 0:
            return
        with stage("scan.hash_agg_kernel"):
            tp = K.ranges_to_tiles(rlen)
            jit.scan_agg(p, rstart, rlen, tp, self._compacts(descs), nrows=r.table.num_rows,
                         hk=hk, htab=table)

    def _topk_request(self, final, fns, order, limit, minmax):
        """(aggregate index, by count, descending, limit) when the query orders by one SUM /
        COUNT aggregate with a small LIMIT (a ``TopKPlan`` can serve it), else None."""
        if not order or limit is None or minmax or not 0 < int(limit) < H_TOPK_K or \
                not HyperspaceConf.run_topk_enabled(self.session.conf):
            return None
        e = order[0].child
        if not isinstance(e, E.Attribute):
            return None
        for agg in final.aggregates:
            a = agg if isinstance(agg, E.Attribute) else agg.to_attribute()
            if a.expr_id != e.expr_id:
                continue
            inner = agg.child if isinstance(agg, E.Alias) else agg
            if not isinstance(inner, (E.Sum, E.Count)):
                return None
            i = next((k for k, fn in enumerate(fns) if fn is inner), None)
            if i is None:
                return None
            return (i, isinstance(inner, E.Count), not order[0].ascending, int(limit))
        return None

    def _topk_plan(self, req, hk, A: int):
        """The cached TopKPlan of a request (buffers reused across queries), or None when the
        order aggregate keeps its own non-null count (a NULL sum has no order value there)."""
        from . import hash_agg as H
        i, by_count, desc, limit = req
        if (hk.own_counts[i] and not by_count) or any(c.nullable for c in hk.cols):
            return None
        plans = self.__dict__.setdefault("_tkplans", {})
        K = 16 if limit <= 16 else 32
        key = (i, by_count, desc, A, K)
        tk = plans.get(key)
        if tk is None:
            tk = plans[key] = H.TopKPlan(i, by_count, desc, A, K)
        return tk

    def _fd_device(self, hk, right: DRel, rk, fd) -> Optional[dict]:
        """The device functional-dependency lookup of run top-K candidates
        (``TopKPlan.gather``'s ``fd``): a single non-null integer key column and at most
        ``TopKPlan.FD_COLS`` fixed-width right columns; None otherwise (``_fd_lookup``)."""
        from . import hash_agg as H
        if len(hk.cols) != 1 or hk.mode not in ("packed", "raw_int") or len(fd[1]) > \
                H.TopKPlan.FD_COLS:
            return None
        c = hk.cols[0]
        if c.kind != "int" or c.nullable or c.dictionary is not None:
            return None
        key = right.col(rk)
        if key.hs_type not in (NL.I8, NL.I16, NL.I32, NL.I64) or key.valid is not None or \
                right.table.bucket_offsets is None:
            return None
        cols = [right.col(a) for a in fd[1]]
        if any(x.offsets is not None for x in cols):
            return None
        raw = hk.mode == "raw_int"
        mask = ((1 << c.bits) - 1) if c.bits < 64 else (1 << 64) - 1
        return {"raw": raw, "lo": 0 if raw else int(c.lo), "shift": 0 if raw else int(c.shift),
                "mask": mask, "key": key, "off": right.table.bucket_offsets,
                "nb": len(right.table.bucket_offsets_host) - 1, "cols": cols}

    def _topk_fast(self, tk, groups, hk, A: int, limit: int, fdd: Optional[dict] = None):
        """(status, host group arrays, table groups) of a run top-K query from one packed copy
        (``TopKPlan.gather``): "ok" with the top-``limit`` candidates of the slots and the
        table (split keys); "over" when the table overflowed (grow and re-run); "exact" when
        the largest value the slots do not hold reaches the k-th best value (a dropped tie is
        possible) or ties of the k-th value overflow the copy (the caller re-runs exactly)."""
        i = tk.agg
        cs = i if hk.own_counts[i] else (A - 1 if hk.need_star else -1)
        r = tk.unpack(tk.gather(groups, cs, limit, fdd), len(fdd["cols"]) if fdd else 0)
        if r["over"]:
            return "over", None, r["G"]
        host = r["host"]
        if host is None:
            return "exact", None, r["G"]
        n = len(host["keys"])
        if r["empty"] and n < limit:
            return "exact", None, r["G"]     # a live entry may share the empty pattern
        if n >= limit:
            vals = np.sort(tk.image(host["sums"], host["cnts"]))[::-1]
            kth = float(vals[limit - 1])
        else:
            kth = -np.inf
        self.metrics["run_topk_guard"] = (float(r["bound"]), kth, n, r["G"])
        if r["bound"] >= kth:
            return "exact", None, r["G"]
        if "fd" in r:
            host["fd"] = r["fd"]
        return "ok", host, r["G"]

    def _hash_prep_get(self, final, order, limit):
        """The kept setup of a hash-mode aggregate node submitted before, while its tables are
        resident (``_HashPrep``), or None."""
        hp = self.__dict__.get("_hash_preps", {}).get(id(final))
        if hp is None or hp.final is not final or hp.order is not order or hp.limit != limit \
                or hp.placement != self._placement_tag() or hp.epoch != self.cache.epoch or \
                not all(self._holds(t) for t in hp.tables):
            return None
        return hp

    def _hash_prep_put(self, final, order, limit, node, launches, setup):
        """Keep a hash-mode join aggregate's setup for its next submission: one join launch
        over resident tables (no bucket-union parts, no computed columns)."""
        if len(launches) != 1 or launches[0][0] != "join":
            return None
        _, a, b = launches[0]
        if a.parts or b.parts or a.extra or b.extra or a.split or b.split or \
                getattr(a.table, "_hs_cache_key", None) is None or \
                getattr(b.table, "_hs_cache_key", None) is None:
            return None
        preps = self.__dict__.setdefault("_hash_preps", {})
        if len(preps) > 64:
            preps.clear()
        hp = _HashPrep(final, order, limit, node, (a.table, b.table), setup,
                       self._placement_tag(), self.cache.epoch)
        preps[id(final)] = hp
        return hp

    def _join_hash_pair(self, node, left: DRel, right: DRel, lk, rk, fns, grouping, doms,
                        table, hk_box, tk_req=None, tk_box=None, prep=None) -> None:
        lkey = prep.literal_key(tk_req) if prep is not None else None
        low = prep.lowered.get(lkey) if lkey is not None else None
        if low is not None:
            # this literal vector was lowered before: bind nothing, launch
            jp, hk, nspecs, comp, rstart, rlen, rbk, left, right, lk, rk, empty = low
            if not hk_box:
                hk_box.append(hk)
            if empty:
                return
            tk = self._topk_plan(tk_req, hk, nspecs) if tk_req is not None else None
            if tk is not None:
                tk.used = False
                tk_box.append(tk)
            fr = getattr(left.table, "_full_ranges", None)
            with stage("join.hash_agg_kernel"):
                jit.merge_join_agg(jp, rstart, rlen, rbk, right.table.bucket_offsets, comp,
                                   nrows=left.table.num_rows,
                                   cache_spans=fr is not None and rstart is fr[0],
                                   rdup=jit.key_has_dups(right.col(rk)), hk=hk, htab=table, tk=tk,
                                   record=HyperspaceConf.join_index_enabled(self.session.conf))
            return
        if right.table.num_rows * 64 < left.table.num_rows:
            left, right, lk, rk = right, left, rk, lk
        implied: set = set()
        probed = self._probe_ranges(left, right, lk, rk)
        if probed is None:
            probed = self._domain_pruned_ranges(left, right, lk, rk)
        if probed is not None:
            rstart, rlen, rbk = probed
        else:
            rstart, rlen, rbk = self._ranges(left, left.conds, implied)
        jp, col_info, descs, keep = self._join_params(
            left, right, lk, rk, node.condition,
            lconds=[c for c in left.conds if id(c) not in implied])
        specs = self._agg_specs(fns, col_info)
        hk = self._hash_keyplan(grouping, col_info, fns, doms, specs, descs)
        if not hk_box:
            hk_box.append(hk)
        jp.group_col, jp.num_groups, jp.group_base = -1, 1, 0
        for s, c in descs.items():
            jp.cols[s] = c.desc()
        for i, a in enumerate(specs):
            jp.aggs[i] = a
        jp.naggs = len(specs)
        if keep[0].always_false or keep[1].always_false or left.table.num_rows == 0 or \
                right.table.num_rows == 0:
            if lkey is not None:
                prep.keep_lowered(lkey, (jp, hk, len(specs), None, None, None, None, left, right,
                                         lk, rk, True))
            return
        comp = self._compacts(descs)
        if not jit.merge_join_ok(jp, comp, right.table.num_rows, left.table.num_rows):
            raise Unsupported("hash aggregate over a join the merge-join kernel cannot run")
        if lkey is not None:
            prep.keep_lowered(lkey, (jp, hk, len(specs), comp, rstart, rlen, rbk, left, right,
                                     lk, rk, False))
        fr = getattr(left.table, "_full_ranges", None)
        tk = self._topk_plan(tk_req, hk, len(specs)) if tk_req is not None else None
        if tk is not None:
            tk.used = False
            tk_box.append(tk)
        with stage("join.hash_agg_kernel"):
            jit.merge_join_agg(jp, rstart, rlen, rbk, right.table.bucket_offsets, comp,
                               nrows=left.table.num_rows,
                               cache_spans=fr is not None and rstart is fr[0],
                               rdup=jit.key_has_dups(right.col(rk)), hk=hk, htab=table, tk=tk,
                               record=HyperspaceConf.join_index_enabled(self.session.conf))

    def _hash_combine_ranks(self, d, groups, G: int, A: int, minmax: bool):
        """Every rank's groups to every rank (one variable-size all-gather of packed rows, no
        pickling), merged in a device table: ranks may share groups (any key not led by the
        bucket key)."""
        from . import hash_agg as H
        with stage("hagg.combine_ranks"):
            host = groups.to_host(G)
            parts = [host["keys"].view(np.int64).reshape(G, 1),
                     host["nulls"].astype(np.int64).reshape(G, 1),
                     host["sums"].view(np.int64), host["cnts"],
                     host["mins"].view(np.int64), host["maxs"].view(np.int64)]
            rows = np.ascontiguousarray(np.concatenate(parts, axis=1)) if G else \
                np.zeros((0, 2 + 4 * A), np.int64)
            allr = d.all_gather_rows(rows)
            n = allr.shape[0]
            if n == 0:
                return groups, 0

            def col(j):
                return np.ascontiguousarray(allr[:, 2 + j * A: 2 + (j + 1) * A])
            merged_in = H.Groups.from_host(
                {"keys": allr[:, 0].copy().view(np.uint64), "nulls": allr[:, 1].astype(np.uint8),
                 "sums": col(0).view(np.float64), "cnts": col(1),
                 "mins": col(2).view(np.float64), "maxs": col(3).view(np.float64)},
                A, minmax, self.device)
            M = H.next_pow2(max(H.MIN_SLOTS, 2 * n))
            table = self.htables.get(M, A, minmax, self.device)
            g = merged_in
            NL.check(NL.lib().hs_hagg_merge(NL.ptr(g.keys), NL.ptr(g.nulls), NL.ptr(g.sums),
                                            NL.ptr(g.cnts), NL.ptr(g.mins), NL.ptr(g.maxs), n,
                                            g.cap, NL.ptr(table.keys), NL.ptr(table.sums),
                                            NL.ptr(table.cnts), NL.ptr(table.mins),
                                            NL.ptr(table.maxs), M, A, NL.ptr(table.flag),
                                            NL.stream_ptr()), "hs_hagg_merge")
            merged = table.extract(A - 1)
            Gm, over = merged.count()
            if over:
                raise Unsupported("rank merge table overflow")
            return merged, Gm

    def _topk_source(self, final, fns, grouping, hk, order, limit, G):
        """The device top-k image of the primary ORDER BY key, or None (host sort of all)."""
        from . import hash_agg as H
        if not order or limit is None or G <= max(TOPK_MIN_GROUPS, 4 * int(limit)) or \
                int(limit) > 1024 or int(limit) <= 0:
            return None
        o = order[0]
        e = o.child
        if not isinstance(e, E.Attribute):
            return None
        desc = not o.ascending
        A = len(fns) + 1
        for agg in final.aggregates:
            a = agg if isinstance(agg, E.Attribute) else agg.to_attribute()
            if a.expr_id != e.expr_id:
                continue
            inner = agg.child if isinstance(agg, E.Alias) else agg
            if isinstance(inner, E.AggregateFunction):
                i = next(k for k, fn in enumerate(fns) if fn is inner)
                cs = i if hk.own_counts[i] else (A - 1 if hk.need_star else -1)
                src = {E.Sum: H.SRC_SUM, E.Count: H.SRC_COUNT, E.Min: H.SRC_MIN,
                       E.Max: H.SRC_MAX, E.Avg: H.SRC_AVG}.get(type(inner))
                if src is None:
                    return None
                return H.OrderSource(src, i, cs, desc=desc)
            if isinstance(inner, E.Attribute):
                e = inner
                break
            return None
        for j, g in enumerate(grouping):
            if g.expr_id != e.expr_id:
                continue
            c = hk.cols[j]
            if hk.mode == "raw_int":
                return H.OrderSource(H.SRC_RAWINT, desc=desc)
            if hk.mode == "raw_float":
                return H.OrderSource(H.SRC_RAWFLT, desc=desc)
            if c.kind == "f32":
                return None
            mask = (1 << c.bits) - 1 if c.bits < 64 else (1 << 64) - 1
            return H.OrderSource(H.SRC_KEYFIELD, shift=c.shift, mask=mask,
                                 nullable=c.nullable, desc=desc)
        return None

    def _hash_table_out(self, final, fns, grouping, hk, host, A, extra=None) -> pa.Table:
        """Result table of a hash-mode aggregate from its host group arrays (vectorized
        finalize; arithmetic over aggregates with pyarrow.compute).  ``extra(gmap, host)`` adds
        group columns not in the key (``_fd_grouping``)."""
        G = 0 if host is None else len(host["keys"])
        if G and hk is not None and not hk.need_star:
            host["cnts"][:, A - 1] = 1     # COUNT(*) not accumulated: every group has rows
        gmap = {}
        if hk is not None and G:
            for g, arr in zip(grouping, hk.unpack(host["keys"], host["nulls"])):
                gmap[g.expr_id] = arr
        else:
            for g in grouping:
                gmap[g.expr_id] = pa.array([], type=g.data_type)
        if extra is not None:
            extra(gmap, host)
        vals = {}
        for i, fn in enumerate(fns):
            if G:
                cnt = host["cnts"][:, i] if (hk.own_counts[i]) else host["cnts"][:, A - 1]
                vals[id(fn)] = _finalize_array(fn, host["sums"][:, i], cnt, host["mins"][:, i],
                                               host["maxs"][:, i])
            else:
                vals[id(fn)] = pa.array([], type=fn.data_type)
        arrays = []
        for e, a in zip(final.aggregates, final.output):
            arr = _eval_vec(e.child if isinstance(e, E.Alias) else e, vals, gmap, G)
            if not arr.type.equals(a.data_type):
                try:
                    arr = arr.cast(a.data_type)
                except (pa.ArrowInvalid, pa.ArrowNotImplementedError):
                    pass
            arrays.append(arr)
        return arrow_table(arrays, [a.name for a in final.output])
