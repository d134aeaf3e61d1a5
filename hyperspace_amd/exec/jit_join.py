"""Join kernel generators (``exec/jit.py``'s code generation for the join family): the generic
tiled join aggregate (``gen_join_agg``), the sort-merge join aggregate over co-located buckets
(``gen_merge_join_agg``: 32-bit merge images, sparse match lists, the run-keyed form over a left
key's run-length encoding, hash-mode GROUP BY), their launch wrappers and span records.  Shared
code-generation helpers and the kernel tunables stay in ``exec/jit.py`` (``J``)."""
from __future__ import annotations

import ctypes as C
import re
import struct
from typing import Dict, List, Optional, Tuple

from ..ops import _lib as NL


def merge_join_shape(p: NL.JoinParams, compacts=None, hk=None) -> tuple:
    cols = tuple(sorted(J._col_specs(p, compacts).items()))
    preds = tuple((p.preds[k].kind, p.preds[k].op, p.preds[k].col, p.preds[k].col2,
                   p.preds[k].group) for k in range(p.npreds))
    aggs = tuple((p.aggs[i].kind, p.aggs[i].nterms, tuple(p.aggs[i].col[:p.aggs[i].nterms]))
                 for i in range(p.naggs))
    return ("merge_join_agg", cols, preds, p.nlp, aggs, p.group_col, p.lkey, p.rkey,
            p.key_is_float, J.MJ_ITEMS, J.MJ_LDS_KEYS, J.MJ_STEPS, J.BLOCK, J.WAVE_SYNC,
            _key32_frame(p, compacts) is not None, J.MJ_STAGE_UNROLL, J.MJ_DBUF, J.MJ_PREFETCH,
            J.MJ_BLOCK, J.MJ_EAGER, J.MJ_SPARSE, J.MJ_HASH_LANEMAJOR, J.MJ_RPF and not J.MJ_PREFETCH, J.MJ_KEY16,
            hk.shape() if hk is not None else None, J.MJ_RUNS, J.MJ_RUNS_ITEMS, J.MJ_RUNS_PREFETCH)


def key_has_dups(col) -> bool:
    """Whether a sorted key column (a join's right side) repeats a non-null key: equal keys hash
    to one bucket, so they are adjacent.  Float keys are assumed to (NaN / -0.0 images).  Cached
    on the column (one device sync per table)."""
    d = getattr(col, "dupkeys", None)
    if d is None:
        x = col.data
        if col.is_float:
            d = True
        elif x.numel() < 2:
            d = False
        else:
            eq = x[1:] == x[:-1]
            if col.valid is not None:
                eq &= (col.valid[1:] != 0) & (col.valid[:-1] != 0)
            d = bool(eq.any().item())
        col.dupkeys = d
    return d


def _slots_of(pred) -> List[int]:
    return J._pred_slots([(0, pred)])


def _key32_frame(p: NL.JoinParams, compacts) -> Optional[Tuple[int, int, int]]:
    """32-bit merge keys: (lo, span, code offset) when the left key is an integer column with a
    compact form whose value range [lo, lo + span] leaves room for the two out-of-range images
    (span <= 2^32 - 3).  Left image = value - lo + 1 = code + (base - lo + 1), in [1, 2^32 - 2];
    a right value maps to the same image, or to 0 / 2^32 - 1 outside the left range (never
    equal to a left image, order kept), so merges compare 32-bit words."""
    if p.key_is_float or not J.MJ_KEY32:
        return None
    c = (compacts or {}).get(p.lkey)
    if c is None or c.scale is not None or getattr(c, "lo", None) is None:
        return None
    span = int(c.hi) - int(c.lo)
    if span > (1 << 32) - 3:
        return None
    return int(c.lo), span, int(c.base) - int(c.lo) + 1


def _deferred_append(NI: int, ind: str, pass_fmt: str, row_fmt: str, j_fmt: str) -> List[str]:
    """Append this thread's passing (row, j) pairs to its wavefront's LDS list (absolute int32
    rows); ``wcnt`` is the wave-uniform list length.  Failing lanes write a private dump slot,
    so the appends are branch-free."""
    b = []
    for it in range(NI):
        b += [f"{ind}{{ const bool pz = {pass_fmt.format(it=it)}; const u64 bm = __ballot(pz);",
              f"{ind}  const int wp = pz ? wcnt + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(bm >> 32), "
              f"__builtin_amdgcn_mbcnt_lo((unsigned)bm, 0u)) : DUMP + cln;",
              f"{ind}  lrow_s[wv][wp] = (int)({row_fmt.format(it=it)}); "
              f"lj_s[wv][wp] = (int)({j_fmt.format(it=it)});",
              f"{ind}  wcnt += __popcll(bm); }}"]
    return b


def _sparse_append(NI: int, ind: str, word: str, j_fmt: str, drain=()) -> List[str]:
    """``_deferred_append`` for sparse matches: the thread's match bits ``word`` are appended
    one set bit per round, for as many rounds as the wavefront's busiest lane needs (a join
    keeping a few percent of its rows: one or two rounds instead of NI).  The item's row is
    ``g0 + it``; its match index comes from a select chain over the per-item registers."""
    b = [f"{ind}{{ unsigned pend = {word};",
         f"{ind}  while (__any(pend != 0u)) {{",
         f"{ind}    const bool has = pend != 0u;",
         f"{ind}    const int it = has ? __builtin_ctz(pend) : 0;",
         f"{ind}    pend &= pend - 1u;",
         f"{ind}    int jv = {j_fmt.format(it=0)};"]
    for it in range(1, NI):
        b.append(f"{ind}    jv = it == {it} ? {j_fmt.format(it=it)} : jv;")
    b += [f"{ind}    const u64 bm = __ballot(has);",
          f"{ind}    const int wp = has ? wcnt + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(bm >> 32), "
          f"__builtin_amdgcn_mbcnt_lo((unsigned)bm, 0u)) : DUMP + cln;",
          f"{ind}    lrow_s[wv][wp] = (int)(g0 + it); lj_s[wv][wp] = (int)(ss + jv);",
          f"{ind}    wcnt += __popcll(bm);"] + list(drain) + [
          f"{ind}  }}",
          f"{ind}}}"]
    return b


def _lanemajor_append(NI: int, ind: str, word: str, j_fmt: str) -> List[str]:
    """Append the thread's matches (bits of ``word``) to the wavefront's list in row order:
    lane t's matches go after those of lanes < t (one wave prefix sum of the match counts), so a
    batch of 64 list entries is 64 consecutive matches of the tile."""
    b = [f"{ind}{{ unsigned pend = {word};",
         f"{ind}  const int mc = __popc(pend);",
         f"{ind}  int mi = mc;",
         f"{ind}  for (int o = 1; o < 64; o <<= 1) {{ const int y = __shfl_up(mi, (unsigned)o, 64); "
         f"if (cln >= o) mi += y; }}",
         f"{ind}  int wp = wcnt + mi - mc;",
         f"{ind}  const int mt = __shfl(mi, 63, 64);",
         f"{ind}  while (pend != 0u) {{",
         f"{ind}    const int it = __builtin_ctz(pend);",
         f"{ind}    pend &= pend - 1u;",
         f"{ind}    int jv = {j_fmt.format(it=0)};"]
    for it in range(1, NI):
        b.append(f"{ind}    jv = it == {it} ? {j_fmt.format(it=it)} : jv;")
    b += [f"{ind}    lrow_s[wv][wp] = (int)(g0 + it); lj_s[wv][wp] = (int)(ss + jv); ++wp;",
          f"{ind}  }}",
          f"{ind}  wcnt += mt;",
          f"{ind}}}"]
    return b


def _deferred_drain(args, cols, split, approx, aggs, grouped, group_col, allslots, ind: str,
                    final: bool, hk=None) -> List[str]:
    """Aggregate full 64-entry batches from the top of the wavefront's list (``final``: every
    remaining entry): the aggregate inputs are gathered once per 64 passing rows, all lanes
    active, instead of once per tile."""
    cond = "wcnt > 0" if final else "wcnt >= 64"
    b = [f"{ind}{J._wave_sync()}",
         f"{ind}while ({cond}) {{",
         f"{ind}  const int cb = wcnt > 64 ? wcnt - 64 : 0;",
         f"{ind}  const int ce = cb + cln;",
         f"{ind}  bool cok = ce < wcnt;",
         f"{ind}  const i64 crow = (i64)lrow_s[wv][cok ? ce : cb];",
         f"{ind}  const i64 cj = (i64)lj_s[wv][cok ? ce : cb];"]
    ind2 = ind + "  "
    g = J._Gen(args, cols, split, ("crow", "cj"), approx, True)
    tail = list(dict.fromkeys(J._agg_slots(aggs) + ([group_col] if grouped else []) +
                              (hk.slots if hk is not None else [])))
    for sl in tail:
        J._uload(g, sl, "c", b, ind2)
    gvar = "gic"
    if grouped:
        base = args.add("q", "group_base", "long long")
        ng = args.add("q", "num_groups", "long long")
        b.append(f"{ind2}const i64 glc = (i64){J._rename(f'x{group_col}', allslots, 'c')} - {base};")
        b.append(f"{ind2}cok = cok && {J._rename(g.ok(group_col), allslots, 'c')} && "
                 f"glc >= 0 && glc < {ng};")
        b.append(f"{ind2}const int {gvar} = cok ? (int)glc : 0;")
    if hk is not None:
        b += [J._rename(x, allslots, "c") for x in J.JH._hash_accumulate(g, aggs, hk, "cok", ind2)]
    else:
        b += [J._rename(x, allslots, "c") for x in J._accumulate(g, aggs, grouped, "cok", gvar, ind2)]
    b += [f"{ind2}wcnt = cb;",
          f"{ind2}{J._wave_sync()}",
          f"{ind}}}"]
    return b


def _mj_items(runs: bool) -> int:
    """Rows per thread of the vectorized merge join: the run-keyed form does little work per row
    and takes longer tiles (MJ_RUNS_ITEMS); ``profiles/mj_micro_r4*.jsonl``."""
    return J.MJ_RUNS_ITEMS if runs and J.MJ_RUNS_ITEMS else J.MJ_ITEMS


def _is_runs(compacts, slot: int) -> bool:
    c = (compacts or {}).get(slot)
    return c is not None and c.signature()[2:3] == ("runs",)


def gen_merge_join_agg(p: NL.JoinParams, compacts=None, hk=None) -> J.Kernel:
    """Co-located sort-merge join + aggregate, re-matching keys every query (no cached join
    index).  Left tiles are ``BLOCK * MJ_ITEMS`` rows of one bucket range, aligned so each thread
    owns ``MJ_ITEMS`` consecutive rows read with aligned vector loads; the tile's right key span
    (``hs_join_spans_sampled``, align = MJ_ITEMS) is staged in LDS.  Per tile:

    1. stage: right key images (32-bit in the left key's frame when ``_key32_frame`` allows,
       else order-preserving u64; nulls as the minimum) and one pass byte per right row — the
       right side's own predicates are evaluated once per right row here, not once per match;
    2. stream: the left key + left predicate columns of the thread's rows (vector loads);
    3. merge: one LDS binary search for the thread's first passing key, then a branch-free walk
       of MJ_STEPS key steps per row (keys ascend through the thread's rows; an FK join moves 0
       or 1 key per row); threads whose walk falls short take a general loop;
    4. tail: passing (row, match) pairs go to per-wavefront LDS lists and the aggregate inputs
       are loaded only for them (``_compacted_tail``); right tables with duplicate keys
       (``a.rdup``) repeat 3-4 for the next equal key until no lane has one.

    The kernel is VALU-issue bound, so the per-row work is kept to a few 32-bit operations
    (profiles/pmc_merge_join_r2.txt).  Spans longer than MJ_LDS_KEYS (many right rows per left
    tile) are searched in HBM.  Reference: the bucketed SortMergeJoin plans of JoinIndexRule
    (JoinIndexRule.scala:63-69), which re-match keys on every query."""
    NI = _mj_items(_is_runs(compacts, p.lkey))  # noqa: N806
    BLOCK = J.MJ_BLOCK  # noqa: N806 — 64: one wavefront per workgroup, no block barriers
    T = BLOCK * NI  # noqa: N806
    LK = J.MJ_LDS_KEYS  # noqa: N806
    args = J.Args()
    for n, ct in (("rstart", "const long long*"), ("rlen", "const long long*"),
                  ("tile_prefix", "const long long*"), ("spans", "const long long*")):
        args.add("p", n, ct)
    args.add("q", "R", "long long")
    args.add("q", "nrows", "long long")
    args.add("q", "rdup", "long long")
    J._common_args(args)
    cols = J._col_specs(p, compacts)
    split = 8
    fl = bool(p.key_is_float)
    lk, rk = p.lkey, p.rkey
    k32 = _key32_frame(p, compacts) is not None
    KT = "unsigned" if k32 else "u64"  # noqa: N806
    KMAX = "0xFFFFFFFFu" if k32 else "~0ull"  # noqa: N806
    if k32:
        args.add("q", "KLO", "long long")
        args.add("q", "KSP", "long long")
        args.add("q", "KOF", "long long")
    lenc = cols[lk][2]
    runs = k32 and lenc is not None and len(lenc) > 2 and lenc[2] == "runs"
    if runs:
        assert 64 % NI == 0 and T <= (1 << 16)
        args.add("p", "TR", "const int*")
        args.add("p", f"RK{lk}", "const int*")
        args.add("p", f"GM{lk}", "const unsigned long long*")
        args.add("p", f"GR{lk}", "const int*")
    lpreds = [(k, p.preds[k]) for k in range(p.nlp)]
    rpreds = [(k, p.preds[k]) for k in range(p.nlp, p.npreds)]
    ronly = [(k, q) for k, q in rpreds if all(x >= split for x in _slots_of(q))]
    mixed = [(k, q) for k, q in rpreds if (k, q) not in ronly]
    aggs = [p.aggs[i] for i in range(p.naggs)]
    grouped = p.group_col >= 0
    assert not (grouped and hk is not None)
    hslots = hk.slots if hk is not None else []
    mixed_left = [x for x in J._pred_slots(mixed) if x < split]
    first = list(dict.fromkeys(([] if runs else [lk]) + J._pred_slots(lpreds) + mixed_left))
    ronly_slots = [x for x in J._pred_slots(ronly)]
    mixed_right = [x for x in J._pred_slots(mixed) if x >= split]
    stage_slots = list(dict.fromkeys([rk] + ronly_slots))
    # eager tail: the aggregate inputs of the left side stream with the tile (vector loads) and
    # the right side's are staged in LDS with the span, so a match accumulates at once - no
    # deferred (row, j) lists (20 KB of LDS per block) and no dependent gathers
    tail_slots = list(dict.fromkeys(J._agg_slots(aggs) + ([p.group_col] if grouped else [])))
    eager = J.MJ_EAGER and hk is None
    rtail = [x for x in tail_slots if x >= split] if eager else []
    if eager:
        first = list(dict.fromkeys(first + [x for x in tail_slots if x < split]))
    allslots = list(dict.fromkeys(first + stage_slots + mixed_right + J._agg_slots(aggs) +
                                  ([p.group_col] if grouped else []) + hslots))
    approx = J._sum_only_slots(lpreds + rpreds, aggs, p.group_col, cols) - {lk, rk} - set(hslots)
    ind = "    "
    g1 = J._Gen(args, cols, split, ("row0", "row0"), approx, True)
    b: List[str] = []
    b += J._acc_decls(aggs, grouped, args)
    W = BLOCK // 64  # noqa: N806
    # list entries: < 64 carried over + one round's appends (all NI items per round, or one
    # item per round with the sparse appends, which drain between rounds)
    lanemajor = hk is not None and J.MJ_HASH_LANEMAJOR
    CAP = 128 if (J.MJ_SPARSE and not lanemajor) else 64 * NI + 64  # noqa: N806
    NB = 2 if J.MJ_DBUF else 1  # noqa: N806
    b += [f"  __shared__ {KT} skeys_[{NB}][{LK + 1}]; __shared__ unsigned char spass_[{NB}][{LK}];",
          "  const int cln = threadIdx.x & 63, wv = threadIdx.x >> 6;"]
    if runs:
        # the tile's run keys (32-bit images), overwritten in place by each run's span match
        b.append(f"  __shared__ unsigned lrk_[{T}];")
    if eager and grouped:
        b += _run_decls(aggs)
    if eager:
        for x in rtail:
            b.append(f"  __shared__ {J._CTYPE[cols[x][0]]} stv{x}_[{NB}][{LK}];")
            if cols[x][1]:
                b.append(f"  __shared__ unsigned char stn{x}_[{NB}][{LK}];")
    else:
        b += [f"  constexpr int DUMP = {CAP};",
              f"  __shared__ int lrow_s[{W}][{CAP + 64}]; __shared__ int lj_s[{W}][{CAP + 64}];",
              "  int wcnt = 0;   // wavefront-uniform length of this wavefront's (row, j) list"]
    rkv = J._valid_expr(g1, rk, "{r}")

    def rimg(val: str) -> str:
        """Merge image of a right key value."""
        if not k32:
            return J._key_expr(val, fl)
        return (f"({{ const i64 d_ = (i64)({val}) - a.KLO; "
                f"d_ < 0 ? 0u : (d_ > a.KSP ? 0xFFFFFFFFu : (unsigned)(d_ + 1)); }})")

    k16 = k32 and not runs and cols[lk][2] is not None and len(cols[lk][2]) > 2
    if k16:
        args.add("p", f"G{lk}", "const int*")
        args.add("p", f"W{lk}", "const int*")

    def limg(it: int) -> str:
        """Merge image of left item ``it`` (grouped 16-bit keys: the thread's 8-aligned rows lie
        in one 64-row group, whose base ``gb_`` is loaded once per tile)."""
        if not k32:
            return J._key_expr(f"x{lk}_{it}", fl)
        if k16:
            return f"(kx_[{it}] + (unsigned)a.KOF)"
        return f"((unsigned)x{lk}v[{it}] + (unsigned)a.KOF)"

    U = max(1, J.MJ_STAGE_UNROLL)  # noqa: N806
    rpf = J.MJ_RPF and not J.MJ_PREFETCH and not runs
    # run-keyed + software pipelining: tile t+1's span bounds, run window, run masks and left
    # vectors are in flight while tile t stages, matches and drains
    runs_pf = runs and J.MJ_RUNS_PREFETCH
    pf_slots = list(dict.fromkeys(stage_slots + rtail))

    def pf_issue(b: List[str], i2: str, ssv: str, sev: str) -> None:
        """Loads of the first staging round of the span [ssv, sev) into the pk/pn registers."""
        b.append(f"{i2}{{ const int nsq_ = (int)({sev} - {ssv});")
        for u in range(U):
            b.append(f"{i2}  const i64 jq{u}_ = {ssv} + ({u * BLOCK} + (int)threadIdx.x < nsq_ ? "
                     f"{u * BLOCK} + (int)threadIdx.x : 0);")
        for u in range(U):
            for sl in pf_slots:
                b.append(f"{i2}  pk{sl}_{u} = {g1.ptr(sl)}[jq{u}_];")
                if cols[sl][1]:
                    b.append(f"{i2}  pn{sl}_{u} = {g1.vptr(sl)}[jq{u}_];")
        b.append(f"{i2}}}")

    def body(b: List[str], full: bool) -> None:
        if rpf:
            # this tile's span and first staging round came with the previous tile; issue the
            # next tile's now (its span bounds were loaded one tile earlier still)
            b.extend([f"{ind}const i64 ss = ssC, se = seC;"])
            for u in range(U):
                for sl in pf_slots:
                    b.append(f"{ind}const {g1.raw_type(sl)} ck{sl}_{u} = pk{sl}_{u};")
                    if cols[sl][1]:
                        b.append(f"{ind}const unsigned char cn{sl}_{u} = pn{sl}_{u};")
            pf_issue(b, ind, "ssN", "seN")
            b.extend([f"{ind}i64 ssNN = 0, seNN = 0;",
                      f"{ind}if (t + 2 < t1) {{ ssNN = a.spans[4 * (t + 2) + 2]; "
                      f"seNN = a.spans[4 * (t + 2) + 3]; }}"])
        elif not runs_pf:
            b.append(f"{ind}const i64 ss = a.spans[4 * t + 2], se = a.spans[4 * t + 3];")
        if runs and runs_pf:
            # span bounds, run window and run masks came with the previous tile (_vec_tiles)
            b.append(f"{ind}for (int q_ = (int)threadIdx.x; q_ < nl_; q_ += {BLOCK}) "
                     f"lrk_[q_] = (unsigned)a.RK{lk}[ra_ + q_] + (unsigned)a.KOF;")
        elif runs:
            # the tile's runs (hs_tile_runs), the thread's 64-row group run mask / base, and the
            # run keys staged as merge images - loads issued with the right span's staging
            b.extend([f"{ind}const int ra_ = a.TR[2 * t], nl_ = a.TR[2 * t + 1];",
                      f"{ind}const i64 gi_ = (g0 < a.nrows ? g0 : a.nrows - 1) >> 6;",
                      f"{ind}const unsigned long long gm_ = a.GM{lk}[gi_];",
                      f"{ind}const int gr_ = a.GR{lk}[gi_];",
                      f"{ind}for (int q_ = (int)threadIdx.x; q_ < nl_; q_ += {BLOCK}) "
                      f"lrk_[q_] = (unsigned)a.RK{lk}[ra_ + q_] + (unsigned)a.KOF;"])
        b.extend([f"{ind}const int ns = (int)(se - ss);",
                  f"{ind}const bool staged = ns <= {LK};",
                  f"{ind}{KT}* const skeys = skeys_[{'(int)(t & 1)' if NB == 2 else '0'}];",
                  f"{ind}unsigned char* const spass = spass_[{'(int)(t & 1)' if NB == 2 else '0'}];"])
        for x in rtail:
            sel = '(int)(t & 1)' if NB == 2 else '0'
            b.append(f"{ind}{J._CTYPE[cols[x][0]]}* const stv{x} = stv{x}_[{sel}];")
            if cols[x][1]:
                b.append(f"{ind}unsigned char* const stn{x} = stn{x}_[{sel}];")
        # (1) stage the right span: key images + right-only predicate pass bytes; each round
        # issues the loads of U rows per thread before any store (one HBM round trip per round
        # instead of one per row)
        stg = "staged"
        okk_fmt = f"n{rk}_s{{u}}" if cols[rk][1] else "true"

        def stage_stores(i2: str) -> None:
            for u in range(U):
                gs = J._Gen(args, cols, split, (f"jr{u}", f"jr{u}"), approx, True)
                cond = J._rename(gs.cnf(ronly), allslots, f"s{u}")
                okk = okk_fmt.format(u=u)
                b.extend([f"{i2}if (sv{u}) {{ const bool kv = {okk};",
                          f"{i2}  skeys[sq{u}] = kv ? {rimg(f'x{rk}_s{u}')} : ({KT})0;",
                          f"{i2}  spass[sq{u}] = (kv && {cond}) ? 1 : 0;"])
                for x in rtail:
                    b.append(f"{i2}  stv{x}[sq{u}] = x{x}_s{u};")
                    if cols[x][1]:
                        b.append(f"{i2}  stn{x}[sq{u}] = n{x}_s{u} ? 1 : 0;")
                b.append(f"{i2}}}")
        if rpf:
            # round 0 from the prefetched registers
            b.append(f"{ind}if ({stg}) {{")
            for u in range(U):
                b.extend([f"{ind}  const int sq{u} = {u * BLOCK} + (int)threadIdx.x;",
                          f"{ind}  const bool sv{u} = sq{u} < ns;"])
                for sl in pf_slots:
                    J._uload_raw(g1, sl, f"s{u}", f"ck{sl}_{u}", f"cn{sl}_{u}", b, ind + "  ")
            stage_stores(ind + "  ")
            b.append(f"{ind}}}")
        sq0 = BLOCK * U if rpf else 0
        b.extend([f"{ind}if ({stg}) for (int sqb = {sq0}; sqb < ns; sqb += {BLOCK * U}) {{"])
        for u in range(U):
            b.extend([f"{ind}  const int sq{u} = sqb + {u * BLOCK} + (int)threadIdx.x;",
                      f"{ind}  const bool sv{u} = sq{u} < ns;",
                      f"{ind}  const i64 jr{u} = ss + (sv{u} ? sq{u} : 0);"])
        for u in range(U):
            gs = J._Gen(args, cols, split, (f"jr{u}", f"jr{u}"), approx, True)
            for sl in pf_slots:
                J._uload(gs, sl, f"s{u}", b, ind + "  ")
        stage_stores(ind + "  ")
        b.extend([f"{ind}}}",
                  f"{ind}if (staged && threadIdx.x == 0) skeys[ns] = {KMAX};   // walk sentinel"])
        # (2) left stream (raw vector arrays come from the tile loop).  Per-item flags live as
        # bits of one VGPR word each (kvb: key valid, mb: left predicates, mtb: matched): a bool
        # per item would hold a 64-bit SGPR lane mask, and 8 items x 4 flags exhaust the SGPRs
        J._vec_load_slots(b, g1, first, NI, ind)
        if k16:
            # 32-bit codes of the thread's rows: group base + 16-bit code, or (a wide group,
            # one straddling two buckets) the 32-bit codes themselves
            b.append(f"{ind}const int gbi_ = a.G{lk}[(g0 < a.nrows ? g0 : a.nrows - 1) >> 6];")
            b.append(f"{ind}unsigned kx_[{NI}];")
            b.append(f"{ind}" + " ".join(f"kx_[{it}] = (unsigned)gbi_ + (unsigned)x{lk}v[{it}];"
                                         for it in range(NI)))
            b.append(f"{ind}if (gbi_ == (int)0x80000000) {{ " + " ".join(
                f"kx_[{it}] = act{it} ? (unsigned)a.W{lk}[g0 + {it}] : 0u;" for it in range(NI)) +
                " }")
        b.append(f"{ind}unsigned kvb = 0u, mb = 0u;")
        for it in range(NI):
            gi = J._Gen(args, cols, split, (f"row{it}", f"row{it}"), approx, True)
            cond = J._rename(gi.cnf(lpreds), allslots, it)
            okl = f"n{lk}_{it}" if cols[lk][1] and not runs else "true"
            b.append(f"{ind}{{ const bool kv = act{it} && {okl}; kvb |= kv ? {1 << it}u : 0u; "
                     f"mb |= (kv && {cond}) ? {1 << it}u : 0u; }}")
            if not runs:
                b.append(f"{ind}const {KT} k{it} = {limg(it)};")
        b.append(f"{ind}{_block_sync(BLOCK)}")
        if runs:
            _runs_match(b, ind, g1, rk, rkv, rimg, NI, BLOCK)

        def bit(word: str, it: int) -> str:
            return f"(({word} >> {it}) & 1u)"
        # (3) merge (the run-keyed form matched runs above instead)
        if not runs:
            b.append(f"{ind}{KT} kf = {KMAX};")
            for it in reversed(range(NI)):
                b.append(f"{ind}kf = {bit('mb', it)} ? k{it} : kf;")
            b.append(f"{ind}unsigned mtb = 0u;")
            for it in range(NI):
                b.append(f"{ind}int jl{it} = 0;")
            b.extend([f"{ind}bool slow = !staged;",
                      f"{ind}int jw0 = 0;",
                      f"{ind}if (staged) {{",
                      f"{ind}  int lo = 0;",
                      f"{ind}  for (int st = ns > 0 ? (1 << (31 - __builtin_clz(ns))) : 0; st > 0; st >>= 1) {{",
                      f"{ind}    const int c = lo + st; const {KT} sv = skeys[c <= ns ? c - 1 : ns];",
                      f"{ind}    lo = (c <= ns && sv < kf) ? c : lo; }}",
                      f"{ind}  jw0 = lo; int jw = lo; {KT} v = skeys[jw];"])
            for it in range(NI):
                b.append(f"{ind}  {{ const {KT} ke = {bit('kvb', it)} ? k{it} : ({KT})0;")
                for _ in range(J.MJ_STEPS):
                    b.append(f"{ind}    {{ const bool c = v < ke; jw += c ? 1 : 0; v = skeys[jw]; }}")
                b.extend([f"{ind}    slow = slow || v < ke;",
                          f"{ind}    mtb |= ({bit('mb', it)} && v == ke && jw < ns) ? {1 << it}u : 0u; "
                          f"jl{it} = jw; }}"])
            b.append(f"{ind}}}")
            b.extend([f"{ind}if (__any(slow)) {{",
                      f"{ind}  if (slow) {{ int jw = jw0; mtb = 0u;"])
            for it in range(NI):
                b.extend([f"{ind}    if ({bit('mb', it)}) {{ bool hit;",
                          f"{ind}      if (staged) {{ while (jw < ns && skeys[jw] < k{it}) ++jw;",
                          f"{ind}        hit = jw < ns && skeys[jw] == k{it}; jl{it} = jw; }}",
                          f"{ind}      else {{ i64 lo = ss, hi = se;",
                          f"{ind}        while (lo < hi) {{ const i64 md = (lo + hi) >> 1; "
                          f"const bool nv = {rkv.format(r='md')}; "
                          f"if (nv || {rimg(g1.value(rk, 'md'))} < k{it}) lo = md + 1; else hi = md; }}",
                          f"{ind}        hit = lo < se && !({rkv.format(r='lo')}) && "
                          f"{rimg(g1.value(rk, 'lo'))} == k{it}; jl{it} = (int)(lo - ss); }}",
                          f"{ind}      mtb |= hit ? {1 << it}u : 0u;",
                          f"{ind}    }}"])
            b.extend([f"{ind}  }}", f"{ind}}}"])

        # (4) match rounds: right predicates at j, compacted aggregate tail; right tables with
        # duplicate keys (a.rdup) repeat for the next equal key until no lane has one
        def one_round(i2: str) -> None:
            b.append(f"{i2}{{ unsigned pb = mtb;")
            if ronly:
                # run-keyed: a staged span's pass bytes were folded into the run matches
                b.append(f"{i2}if ({'false' if runs else 'staged'}) {{")
                for it in range(NI):
                    b.append(f"{i2}  pb &= spass[{bit('mtb', it)} ? jl{it} : 0] != 0 ? ~0u : ~{1 << it}u;")
                b.append(f"{i2}}} else{' if (!staged)' if runs else ''} {{")
                for it in range(NI):
                    b.append(f"{i2}  {{ const i64 jq{it} = ss + ({bit('mtb', it)} ? jl{it} : 0);")
                    g2 = J._Gen(args, cols, split, (f"row{it}", f"jq{it}"), approx, True)
                    for sl in ronly_slots:
                        J._uload(g2, sl, it, b, i2 + "    ")
                    b.append(f"{i2}    pb &= ({J._rename(g2.cnf(ronly), allslots, it)}) ? ~0u : ~{1 << it}u; }}")
                b.append(f"{i2}}}")
            if mixed:
                for it in range(NI):
                    b.append(f"{i2}{{ const i64 jm{it} = ss + ({bit('pb', it)} ? jl{it} : 0);")
                    g2 = J._Gen(args, cols, split, (f"row{it}", f"jm{it}"), approx, True)
                    for sl in mixed_right:
                        J._uload(g2, sl, f"{it}m", b, i2 + "  ")
                    cond = J._rename(J._rename(g2.cnf(mixed), mixed_right, f"{it}m"), first, it)
                    b.append(f"{i2}  pb &= ({cond}) ? ~0u : ~{1 << it}u; }}")
            if eager:
                b.extend(_eager_tail(args, cols, split, approx, aggs, grouped, p.group_col,
                                     allslots, rtail, NI, i2))
            else:
                drain = _deferred_drain(args, cols, split, approx, aggs, grouped, p.group_col,
                                        allslots, i2 + "    ", final=False, hk=hk)
                if hk is not None and J.MJ_HASH_LANEMAJOR:
                    # hash-mode grouping: matches appended in row order (lane-major), so equal
                    # keys of a batch are adjacent and merge into one probe per run
                    b.extend(_lanemajor_append(NI, i2, "pb", "jl{it}"))
                    b.extend(_deferred_drain(args, cols, split, approx, aggs, grouped,
                                             p.group_col, allslots, i2, final=False, hk=hk))
                elif J.MJ_SPARSE:
                    # drained inside the append rounds: the lists never hold more than 63 + 64
                    # entries, so they take 6 KB of LDS per block instead of 20 KB
                    b.extend(_sparse_append(NI, i2, "pb", "jl{it}", drain))
                else:
                    b.extend(_deferred_append(NI, i2, "((pb >> {it}) & 1u)", "row{it}",
                                              "ss + jl{it}"))
                    b.extend(_deferred_drain(args, cols, split, approx, aggs, grouped,
                                             p.group_col, allslots, i2, final=False, hk=hk))
            b.append(f"{i2}}}")

        one_round(ind)
        if runs:    # unique right keys only (merge_join_agg): no duplicate-key rounds
            if NB == 1:
                b.append(f"{ind}{_block_sync(BLOCK)}")
            return
        b.append(f"{ind}if (a.rdup) while (true) {{")
        i2 = ind + "  "
        for it in range(NI):
            b.extend([f"{i2}if ({bit('mtb', it)}) {{ ++jl{it};",
                      f"{i2}  const bool more = jl{it} < ns && (staged ? skeys[jl{it}] == k{it} : "
                      f"(!({rkv.format(r=f'(ss + jl{it})')}) && "
                      f"{rimg(g1.value(rk, f'(ss + jl{it})'))} == k{it}));",
                      f"{i2}  if (!more) mtb &= ~{1 << it}u; }}"])
        b.append(f"{i2}if (!__any(mtb != 0u)) break;")
        one_round(i2)
        b.append(f"{ind}}}")
        if NB == 1:   # single span buffer: the next tile's staging must wait for this tile
            b.append(f"{ind}{_block_sync(BLOCK)}")
        if rpf:
            b.append(f"{ind}ssC = ssN; seC = seN; ssN = ssNN; seN = seNN;")

    loads = J._vec_loads(g1, first)
    if rpf:
        # the span registers and the first prefetch (tile t0), before the tile loop
        pre: List[str] = ["  i64 ssC = 0, seC = 0, ssN = 0, seN = 0;"]
        for u in range(U):
            for sl in pf_slots:
                pre.append(f"  {g1.raw_type(sl)} pk{sl}_{u} = 0;")
                if cols[sl][1]:
                    pre.append(f"  unsigned char pn{sl}_{u} = 0;")
        pre.append("  if (t0 < t1) { ssC = a.spans[4 * t0 + 2]; seC = a.spans[4 * t0 + 3]; }")
        pre.append("  if (t0 + 1 < t1) { ssN = a.spans[4 * (t0 + 1) + 2]; "
                   "seN = a.spans[4 * (t0 + 1) + 3]; }")
        pf_issue(pre, "  ", "ssC", "seC")
        b += J._TILE_HEAD + pre
    if runs_pf:
        gi = "((G0 < a.nrows ? G0 : a.nrows - 1) >> 6)"
        J._vec_tiles(b, T, NI, ind, loads,
                   [("gm_", "unsigned long long", f"a.GM{lk}[{gi}]"),
                    ("gr_", "int", f"a.GR{lk}[{gi}]")], body,
                   [("ss", "i64", "a.spans[4 * ({t}) + 2]"), ("se", "i64", "a.spans[4 * ({t}) + 3]"),
                    ("ra_", "int", "a.TR[2 * ({t})]"), ("nl_", "int", "a.TR[2 * ({t}) + 1]")])
    elif J.MJ_PREFETCH:
        # software-pipelined: tile t+1's left vectors are in flight during tile t's staging,
        # search and aggregate tail (the kernel waits on memory ~60% of its wave cycles:
        # profiles/pmc_merge_join_r3.txt)
        J._vec_tiles(b, T, NI, ind, loads, [], body)
    else:
        if rpf:
            b += ["  for (i64 t = t0; t < t1; ++t) {",
                  "    while (r + 1 < (int)a.R && a.tile_prefix[r + 1] <= t) ++r;",
                  f"    const i64 off = (t - a.tile_prefix[r]) * {T};"]
            J._vec_rows(b, NI, ind)
        else:
            J._tile_loop(b, T, NI, 1, ind)
        b.append(f"{ind}if (tb0 + {T} <= a.nrows) {{")
        J._vec_issue(b, loads, NI, ind, True)
        body(b, True)
        b.append(f"{ind}}} else {{")
        J._vec_issue(b, loads, NI, ind, False)
        body(b, False)
        b.append(f"{ind}}}")
    b += ["  }"]
    if eager and grouped:
        b += _run_flush(aggs, "  ")
    if not eager:
        b += _deferred_drain(args, cols, split, approx, aggs, grouped, p.group_col, allslots,
                             "  ", final=True, hk=hk)
    if hk is None:
        b += J._flush(aggs, grouped, BLOCK)
    src = (J._PRELUDE + args.struct_src() +
           f'extern "C" __global__ __launch_bounds__({BLOCK}) void hs_jit_merge_join_agg(Args a) {{\n' +
           "\n".join(b) + "\n}\n")
    lds = (len(aggs) * p.num_groups * 32) if grouped else 0
    return J.Kernel(src, "hs_jit_merge_join_agg", args, lds, BLOCK)


def _runs_match(b: List[str], ind: str, g1: "_Gen", rk: int, rkv: str, rimg, NI: int,
                BLOCK: int) -> None:  # noqa: N803
    """Run-keyed merge (MJ_RUNS): each thread matches a contiguous chunk of the tile's runs
    against the staged right span - one LDS binary search for its first run, then a walk (an FK
    join moves one right key per run) - and overwrites each run's key in ``lrk_`` with its span
    index (~0u: no match).  Neighbouring lanes search neighbouring keys, so the search and the
    walk touch neighbouring LDS words.  Each row then reads its run's entry: run = group base +
    popcount of the group's run-start bits up to the row."""
    rv = lambda r: rimg(g1.value(rk, r))  # noqa: E731
    b.extend([f"{ind}{{ const int c_ = (nl_ + {BLOCK - 1}) / {BLOCK};",
              f"{ind}  const int q0_ = (int)threadIdx.x * c_;",
              f"{ind}  const int q1_ = q0_ + c_ < nl_ ? q0_ + c_ : nl_;",
              f"{ind}  if (staged) {{",
              f"{ind}    int j_ = 0;",
              f"{ind}    if (q0_ < q1_) {{ const unsigned key_ = lrk_[q0_]; int lo = 0;",
              f"{ind}      for (int st = ns > 0 ? (1 << (31 - __builtin_clz(ns))) : 0; st > 0; st >>= 1) {{",
              f"{ind}        const int c = lo + st; lo = (c <= ns && skeys[c - 1] < key_) ? c : lo; }}",
              f"{ind}      j_ = lo; }}",
              f"{ind}    for (int q = q0_; q < q1_; ++q) {{",
              f"{ind}      const unsigned key_ = lrk_[q];",
              f"{ind}      if (skeys[j_] < key_) {{ ++j_;",
              f"{ind}        if (skeys[j_] < key_) {{ int lo = j_ + 1, hi = ns;",
              f"{ind}          while (lo < hi) {{ const int m = (lo + hi) >> 1; "
              f"if (skeys[m] < key_) lo = m + 1; else hi = m; }}",
              f"{ind}          j_ = lo; }} }}",
              f"{ind}      lrk_[q] = (j_ < ns && skeys[j_] == key_ && spass[j_]) ? (unsigned)j_ : 0xFFFFFFFFu;",
              f"{ind}    }}",
              f"{ind}  }} else {{",
              f"{ind}    for (int q = q0_; q < q1_; ++q) {{ const unsigned key_ = lrk_[q]; "
              f"i64 lo = ss, hi = se;",
              f"{ind}      while (lo < hi) {{ const i64 md = (lo + hi) >> 1; "
              f"const bool nv = {rkv.format(r='md')}; "
              f"if (nv || {rv('md')} < key_) lo = md + 1; else hi = md; }}",
              f"{ind}      lrk_[q] = (lo < se && !({rkv.format(r='lo')}) && {rv('lo')} == key_) ? "
              f"(unsigned)(lo - ss) : 0xFFFFFFFFu; }}",
              f"{ind}  }}",
              f"{ind}}}",
              f"{ind}__syncthreads();",
              f"{ind}unsigned mtb = 0u;"])
    for it in range(NI):
        b.append(f"{ind}int jl{it} = 0;")
    # the thread's NI rows lie in one 64-row group: their run-start bits, shifted down, fit in
    # 32 bits, so each row's run is the first row's run plus one popcount (no carried chain)
    b.extend([f"{ind}{{ const int sh_ = (int)(g0 & 63);",
              f"{ind}  const int rq0_ = gr_ + (int)__popcll(gm_ & ((2ull << sh_) - 2ull)) - ra_;",
              f"{ind}  const unsigned gl_ = (unsigned)(gm_ >> sh_);",
              f"{ind}  const int rmax_ = nl_ > 0 ? nl_ - 1 : 0;"])
    for it in range(NI):
        rq = "rq0_" if it == 0 else f"(rq0_ + (int)__popc(gl_ & {(2 << it) - 2}u))"
        b.extend([f"{ind}  {{ const int ri_ = min(max({rq}, 0), rmax_);",
                  f"{ind}    const unsigned jm_ = lrk_[ri_];",
                  f"{ind}    const bool h_ = ((mb >> {it}) & 1u) && jm_ != 0xFFFFFFFFu;",
                  f"{ind}    mtb |= h_ ? {1 << it}u : 0u; jl{it} = h_ ? (int)jm_ : 0; }}"])
    b.append(f"{ind}}}")


def _eager_tail(args, cols, split, approx, aggs, grouped, group_col, allslots, rtail, NI: int,
                ind: str) -> List[str]:
    """Merge-join matches of this round (bit ``it`` of ``pb``) accumulated at once: left inputs
    are the tile's registers ``x<s>_<it>``, right inputs come from the staged span (``stv<s>``
    at ``jl<it>``; an unstaged span reads them from HBM)."""
    b = []
    for it in range(NI):
        b.append(f"{ind}{{ bool pe = ((pb >> {it}) & 1u) != 0u; const int je = pe ? jl{it} : 0;")
        gr = J._Gen(args, cols, split, (f"row{it}", "(ss + je)"), approx, True)
        for x in rtail:
            ct = J._CTYPE[cols[x][0]]
            b.append(f"{ind}  const {ct} x{x}_{it} = staged ? stv{x}[je] : {gr.value(x, '(ss + je)')};")
            if cols[x][1]:
                b.append(f"{ind}  const bool n{x}_{it} = staged ? stn{x}[je] != 0 : "
                         f"{gr.vptr(x)}[ss + je] != 0;")
        g = J._Gen(args, cols, split, (f"row{it}", "(ss + je)"), approx, True)
        gvar = f"gi{it}"
        if grouped:
            base = args.add("q", "group_base", "long long")
            ng = args.add("q", "num_groups", "long long")
            b.append(f"{ind}  const i64 gl = (i64){J._rename(f'x{group_col}', allslots, it)} - {base};")
            b.append(f"{ind}  pe = pe && {J._rename(g.ok(group_col), allslots, it)} && "
                     f"gl >= 0 && gl < {ng};")
            b.append(f"{ind}  const int {gvar} = pe ? (int)gl : 0;")
            b += [J._rename(x, allslots, it) for x in _run_accumulate(g, aggs, "pe", gvar,
                                                                    ind + "  ")]
        else:
            b += [J._rename(x, allslots, it) for x in J._accumulate(g, aggs, grouped, "pe", gvar,
                                                                 ind + "  ")]
        b.append(f"{ind}}}")
    return b


def _run_decls(aggs) -> List[str]:
    """Per-thread run accumulators of grouped eager aggregation (``_run_accumulate``)."""
    out = ["  int rg_ = -1;"]
    for i, a in enumerate(aggs):
        out.append(f"  double rs{i}_ = {J._ident(a.kind)}; unsigned long long rc{i}_ = 0ull;")
    return out


def _run_flush(aggs, ind: str) -> List[str]:
    """Add this thread's run (group ``rg_``) to the block's LDS group table."""
    out = [f"{ind}if (rg_ >= 0) {{"]
    for i, a in enumerate(aggs):
        out.append(f"{ind}  if (rc{i}_) {{ const int s = rg_ * NA + {i};")
        if a.kind == NL.AK_MIN:
            out.append(f"{ind}    lds_min(&gmn[s], rs{i}_);")
        elif a.kind == NL.AK_MAX:
            out.append(f"{ind}    lds_max(&gmx[s], rs{i}_);")
        elif a.kind == NL.AK_SUM:
            out.append(f"{ind}    atomicAdd(&gsum[s], rs{i}_);")
        out.append(f"{ind}    atomicAdd(&gcnt[s], rc{i}_); }}")
    out.append(f"{ind}}}")
    return out


def _run_accumulate(gen: J._Gen, aggs, pass_var: str, gvar: str, ind: str) -> List[str]:
    """Grouped accumulation into per-thread registers while consecutive matches of the thread
    stay in one group (sorted / low-cardinality groups: almost always), flushed to the LDS group
    table when the group changes - instead of a wavefront-wide peel per row."""
    out = [f"{ind}if ({pass_var}) {{",
           f"{ind}  if ({gvar} != rg_) {{"]
    out += _run_flush(aggs, ind + "    ")
    out.append(f"{ind}    rg_ = {gvar};")
    for i, a in enumerate(aggs):
        out.append(f"{ind}    rs{i}_ = {J._ident(a.kind)}; rc{i}_ = 0ull;")
    out.append(f"{ind}  }}")
    for i, a in enumerate(aggs):
        v, ok = gen.agg_value(i, a)
        upd = {NL.AK_MIN: f"rs{i}_ = fmin(rs{i}_, (double)({v}));",
               NL.AK_MAX: f"rs{i}_ = fmax(rs{i}_, (double)({v}));"}.get(
            a.kind, f"rs{i}_ += (double)({v});")
        out.append(f"{ind}  if ({ok}) {{ {upd} rc{i}_ += 1ull; }}")
    out.append(f"{ind}}}")
    return out


def _block_sync(block: int) -> str:
    """Workgroup barrier; a one-wavefront workgroup only needs its LDS accesses ordered."""
    return J._wave_sync(True) if block == 64 else "__syncthreads();"


def merge_join_ok(p: NL.JoinParams, compacts=None, rnrows: int = 0, lnrows: int = 0) -> bool:
    """The vectorized merge join needs 16-byte aligned bases of the streamed left columns and
    left / right row indices that fit its int32 aggregate lists."""
    if J.MJ_ITEMS <= 0 or rnrows >= (1 << 31) or lnrows >= (1 << 31):
        return False
    ptrs = []
    slots = [p.lkey] + J._pred_slots([(k, p.preds[k]) for k in range(p.nlp)]) + \
        [x for x in J._pred_slots([(k, p.preds[k]) for k in range(p.nlp, p.npreds)]) if x < 8]
    for s in dict.fromkeys(slots):
        c = (compacts or {}).get(s)
        ptrs.append(c.codes.data_ptr() if c else p.cols[s].data)
        ptrs.append(p.cols[s].valid)
    return J._vec_aligned_ptrs(ptrs)


def merge_join_agg(p: NL.JoinParams, rstart, rlen, rbucket, roff, compacts=None, nrows: int = 0,
                   cache_spans: bool = False, rdup: bool = True, hk=None, htab=None, tk=None,
                   record: bool = False):
    """Sort-merge join + aggregate with ``gen_merge_join_agg`` (same outputs as ``join_agg``);
    ``nrows`` = left table rows; ``rdup`` = the right key column may repeat a key
    (``key_has_dups``).  ``record``: a reused two-phase lowering may keep its key match
    (``jit_runs.TwoPhaseLauncher._record``: a join index in run form) - only where join indexes
    are enabled; otherwise every launch re-matches the keys."""
    runs = None
    if not rdup:
        compacts, runs = _with_runs(p, compacts)
    if hk is None and runs is not None:
        from . import jit_runs
        # over a resident table's cached full ranges the lowering is fixed (as in hash mode
        # below): a caller without a prepared launcher (the co-partitioned semi-join) reuses it
        ck = (id(rstart), id(runs), tuple(p.cols[s].data for s in range(NL.MAX_COLS)),
              merge_join_shape(p, compacts), record) if cache_spans else None
        two = _RUNS_LOWERED.get(ck) if ck is not None else None
        if two is None:
            two = jit_runs.lower(p, rstart, rlen, rbucket, roff, compacts, runs, nrows,
                                 cache_spans, record=record)
            if two is not None and ck is not None:
                if len(_RUNS_LOWERED) >= 8:
                    _RUNS_LOWERED.pop(next(iter(_RUNS_LOWERED)))
                _RUNS_LOWERED[ck] = two
        if two is not None:
            LAST_MJ_LAUNCHER[0] = two
            return two.launch(p)
    if hk is not None and runs is not None and J.MJ_RUNS_HASH:
        from . import jit_runs
        # over a resident table's cached full ranges the lowering (run ranges, tiles, kernels,
        # column slots) is fixed: keep it, keyed by the ranges, the column pointers and the shape
        ck = (id(rstart), id(runs), tuple(p.cols[s].data for s in range(NL.MAX_COLS)),
              merge_join_shape(p, compacts, hk), id(tk),
              tk.shape() if tk is not None else None, record) if cache_spans else None
        two = _RUNS_HASH_LOWERED.get(ck) if ck is not None else None
        if two is None:
            two = jit_runs.lower(p, rstart, rlen, rbucket, roff, compacts, runs, nrows,
                                 cache_spans, hk=hk, tk=tk, record=record)
            if two is not None and ck is not None:
                if len(_RUNS_HASH_LOWERED) >= 8:
                    _RUNS_HASH_LOWERED.pop(next(iter(_RUNS_HASH_LOWERED)))
                _RUNS_HASH_LOWERED[ck] = two
        if two is not None:
            LAST_MJ_PATH[0] = "runs_hash"
            two.launch(p, htab=htab, hk=hk)
            return None
    if hk is not None:
        LAST_MJ_PATH[0] = "hash"
    if hk is None and runs is None:
        compacts = _with_key16(p, compacts)
    NI = _mj_items(runs is not None)  # noqa: N806
    T = J.MJ_BLOCK * NI  # noqa: N806
    GA = p.naggs * (p.num_groups if p.group_col >= 0 else 1)
    dev = rstart.device
    max_tiles = nrows // T + 2 * rstart.numel() + 2
    tp, spans = _join_spans(p, rstart, rlen, rbucket, roff, max_tiles, T, cache_spans, align=NI)
    k = J.kernel_for(merge_join_shape(p, compacts, hk), lambda: gen_merge_join_agg(p, compacts, hk))
    grid = max(1, J.MJ_GRID * 256 // J.MJ_BLOCK)
    tr = _tile_runs(tp, spans, rstart.numel(), runs, max_tiles, cache_spans) \
        if runs is not None else None
    if hk is not None:
        v = {"rstart": rstart.data_ptr(), "rlen": rlen.data_ptr(), "tile_prefix": tp.data_ptr(),
             "spans": spans.data_ptr(), "R": rstart.numel(), "nrows": nrows, "rdup": int(rdup),
             "psum": 0, "pcnt": 0, "pmin": 0, "pmax": 0, "TR": tr.data_ptr() if tr is not None else 0}
        J._fill_common(v, p.cols, [(k_, p.preds[k_]) for k_ in range(p.npreds)],
                     [p.aggs[i] for i in range(p.naggs)], compacts)
        frame = _key32_frame(p, compacts)
        if frame is not None:
            v["KLO"], v["KSP"], v["KOF"] = frame
        v.update(htab.kernel_values())
        v.update(hk.values())
        k.launch(grid, v, NL.stream_ptr(), 0)
        return None
    v = {"rstart": rstart.data_ptr(), "rlen": rlen.data_ptr(), "tile_prefix": tp.data_ptr(),
         "spans": spans.data_ptr(), "R": rstart.numel(), "nrows": nrows, "rdup": int(rdup),
         "num_groups": p.num_groups, "group_base": p.group_base,
         "TR": tr.data_ptr() if tr is not None else 0}
    J._fill_cols(v, p.cols, compacts)
    frame = _key32_frame(p, compacts)
    if frame is not None:
        v["KLO"], v["KSP"], v["KOF"] = frame
    launcher = MergeJoinLauncher(k, grid, GA, GA * 32 if p.group_col >= 0 else 0, v, compacts,
                                 (rstart, rlen, rbucket, roff, tp, spans, tr), dev)
    LAST_MJ_LAUNCHER[0] = launcher
    return launcher.launch(p)


# the launcher merge_join_agg built last (GpuBackend keeps it for the query's next submission)
LAST_MJ_LAUNCHER: list = [None]
# which form the last hash-mode merge join took ("runs_hash" / "hash")
LAST_MJ_PATH: list = [None]
# cached two-phase hash-mode lowerings (merge_join_agg); each holds its ranges / run form, so
# the ids in its key stay valid while it is cached
_RUNS_HASH_LOWERED: Dict[tuple, object] = {}
_RUNS_LOWERED: Dict[tuple, object] = {}


class MergeJoinLauncher:
    """A merge-join aggregate lowered once - generated kernel, tile spans / run windows and the
    column argument slots; ``launch(p)`` fills only the literal-dependent slots (predicate
    values, aggregate terms) of ``p`` and queues the kernel and the partials fold."""
    __slots__ = ("k", "grid", "GA", "shmem", "values", "compacts", "keep", "dev")

    def __init__(self, k, grid, GA, shmem, values, compacts, keep, dev):
        self.k, self.grid, self.GA, self.shmem = k, grid, GA, shmem
        self.values, self.compacts, self.keep, self.dev = values, compacts, keep, dev

    def launch(self, p: NL.JoinParams):
        parts = J._partials(self.grid, self.GA, self.dev)
        v = dict(self.values)
        v.update({"psum": parts[0].data_ptr(), "pcnt": parts[1].data_ptr(),
                  "pmin": parts[2].data_ptr(), "pmax": parts[3].data_ptr()})
        J.fill_preds_aggs(v, [(k_, p.preds[k_]) for k_ in range(p.npreds)],
                        [p.aggs[i] for i in range(p.naggs)], self.compacts)
        self.k.launch(self.grid, v, NL.stream_ptr(), self.shmem)
        return J._final(parts, self.grid, self.GA, self.dev)


def _with_runs(p: NL.JoinParams, compacts):
    """(``compacts`` with the left key's run-length form, that form) when the run-keyed merge
    join applies: a 32-bit-frame left key without nulls whose runs average at least
    ``encoding.MIN_ROWS_PER_RUN`` rows; else (``compacts``, None).  Callers use it only for
    unique right keys."""
    from .encoding import GroupedCompact, key_runs
    ni = _mj_items(True)
    if not (J.MJ_RUNS and ni and 64 % ni == 0) or _key32_frame(p, compacts) is None:
        return compacts, None
    lk = p.lkey
    c = compacts.get(lk)
    if p.cols[lk].valid or c is None or isinstance(c, GroupedCompact):
        return compacts, None
    r = key_runs(c)
    if r is None:
        return compacts, None
    out = dict(compacts)
    out[lk] = r
    return out, r


# (spans id, run form id) -> (spans, run form, per-tile (first run, run count) int32 pairs)
_TRUNS: Dict[tuple, tuple] = {}


def _tile_runs(tp, spans, R: int, rc, max_tiles: int, cache: bool):
    """Per merge-join tile: its first run and run count (csrc/kernels/key_runs.hip)."""
    import torch
    key = (id(spans), id(rc))
    if cache:
        hit = _TRUNS.get(key)
        if hit is not None and hit[0] is spans and hit[1] is rc:
            return hit[2]
    out = torch.empty(2 * max(int(max_tiles), 1), dtype=torch.int32, device=spans.device)
    NL.check(NL.lib().hs_tile_runs(tp.data_ptr(), R, spans.data_ptr(), rc.gmask.data_ptr(),
                                   rc.gruns.data_ptr(), int(max_tiles), out.data_ptr(),
                                   NL.stream_ptr()), "hs_tile_runs")
    if cache:
        if len(_TRUNS) >= 16:
            _TRUNS.pop(next(iter(_TRUNS)))
        _TRUNS[key] = (spans, rc, out)
    return out


def _with_key16(p: NL.JoinParams, compacts):
    """``compacts`` with the left key's grouped 16-bit form (encoding.grouped16) when the merge
    join reads that column only as its 32-bit-frame join key (no validity, no predicate,
    aggregate or group use) and every 64-row group of it spans < 2^16 codes."""
    from .encoding import grouped16
    if not (J.MJ_KEY16 and J.MJ_ITEMS and 64 % J.MJ_ITEMS == 0) or _key32_frame(p, compacts) is None:
        return compacts
    lk = p.lkey
    if p.cols[lk].valid:
        return compacts
    used = set(J._pred_slots([(k, p.preds[k]) for k in range(p.npreds)])) | \
        set(J._agg_slots([p.aggs[i] for i in range(p.naggs)])) | {p.group_col}
    if lk in used:
        return compacts
    g = grouped16(compacts[lk])
    if g is None:
        return compacts
    out = dict(compacts)
    out[lk] = g
    return out


def _sample_offsets(roff):
    """Per-bucket offsets of the right side's sparse key samples (every ``hs_join_sample_stride``
    -th key) and a host bound on their count.  Bucket offsets of a device table never change, so
    this is computed once per right table (keyed by tensor identity, holding a reference)."""
    import torch
    hit = J._SOFF.get(id(roff))
    if hit is not None and hit[0] is roff:
        return hit[1], hit[2]
    stride = NL.lib().hs_join_sample_stride()
    n = roff[1:] - roff[:-1]
    soff = torch.zeros(roff.numel(), dtype=torch.int64, device=roff.device)
    torch.cumsum((n + stride - 1) // stride, 0, out=soff[1:])
    B = roff.numel() - 1
    bound = int(roff[-1].item()) // stride + B  # one sync per right table, then cached
    if len(J._SOFF) > 64:
        J._SOFF.clear()
    J._SOFF[id(roff)] = (roff, soff, bound)
    return soff, bound

# (identity key) -> (refs..., tile_prefix, spans): span records of full-range joins.  Holding the
# range / offset tensors keeps their ids from being reused while the entry lives.
_SPANS: Dict[tuple, tuple] = {}


def _join_spans(p: NL.JoinParams, rstart, rlen, rbucket, roff, max_tiles: int, tile: int,
                cache: bool, align: int = 1):
    """(tile_prefix, spans) of the left ranges: per ``tile``-row tile its (row0, rows, rs, re).
    ``align`` > 1: tiles start at each range's start rounded down to a multiple of ``align``
    (the vectorized merge join), ``max_tiles`` is then a bound on the tile count itself."""
    import torch
    from ..ops import kernels as K
    L = NL.lib()
    lk, rk = p.cols[p.lkey], p.cols[p.rkey]
    key = (id(rstart), id(rlen), id(rbucket), id(roff), lk.data, lk.valid, rk.data, rk.valid,
           int(p.key_is_float), tile, align)
    if cache:
        hit = _SPANS.get(key)
        if hit is not None and hit[0] is rstart and hit[1] is rlen and hit[2] is rbucket \
                and hit[3] is roff:
            return hit[4], hit[5]
    dev = rstart.device
    if align > 1:
        tp = K.ranges_to_tiles(rlen + (rstart & (align - 1)), tile)
        mt = int(max_tiles)
    else:
        tp = K.ranges_to_tiles(rlen, tile)
        mt = (max_tiles * L.hs_join_tile_rows()) // tile + rlen.numel() + 1
    spans = torch.empty(4 * mt, dtype=torch.int64, device=dev)
    soff, bound = _sample_offsets(roff)
    samples = torch.empty(max(bound, 1), dtype=torch.int64, device=dev)
    NL.check(L.hs_join_spans_sampled(C.byref(p), NL.ptr(rstart), NL.ptr(rlen), NL.ptr(rbucket),
                                     NL.ptr(roff), NL.ptr(soff), roff.numel() - 1, bound,
                                     NL.ptr(samples), rstart.numel(), NL.ptr(tp), int(mt),
                                     NL.ptr(spans), tile, int(align), NL.stream_ptr()),
             "hs_join_spans_sampled")
    if cache:
        if len(_SPANS) >= 16:
            _SPANS.pop(next(iter(_SPANS)))
        _SPANS[key] = (rstart, rlen, rbucket, roff, tp, spans)
    return tp, spans


def join_agg_values(p: NL.JoinParams, tile_prefix, spans, parts,
                    compacts=None) -> Dict[str, object]:
    v = {"tile_prefix": tile_prefix.data_ptr(), "R": tile_prefix.numel() - 1,
         "spans": spans.data_ptr(), "psum": parts[0].data_ptr(), "pcnt": parts[1].data_ptr(),
         "pmin": parts[2].data_ptr(), "pmax": parts[3].data_ptr(),
         "num_groups": p.num_groups, "group_base": p.group_base}
    J._fill_common(v, p.cols, [(k, p.preds[k]) for k in range(p.npreds)],
                 [p.aggs[i] for i in range(p.naggs)], compacts)
    return v


__all__ = ['LAST_MJ_LAUNCHER', 'LAST_MJ_PATH', 'MergeJoinLauncher', '_RUNS_HASH_LOWERED',
           '_RUNS_LOWERED',
           '_SPANS', '_TRUNS', '_block_sync', '_deferred_append', '_deferred_drain',
           '_eager_tail', '_is_runs', '_join_spans', '_key32_frame', '_lanemajor_append',
           '_mj_items', '_run_accumulate', '_run_decls', '_run_flush', '_runs_match',
           '_sample_offsets', '_slots_of', '_sparse_append', '_tile_runs', '_with_key16',
           '_with_runs', 'gen_merge_join_agg', 'join_agg_values', 'key_has_dups',
           'merge_join_agg', 'merge_join_ok', 'merge_join_shape']

# jit is imported last: its module body re-exports this module's names when it finishes
from . import jit as J  # noqa: E402
from . import jit_hash as JH  # noqa: E402,F401
