"""Hash-mode GROUP BY and run top-K code emitters for the generated kernels (``exec/jit.py``,
``exec/jit_runs.py``): the segmented shuffle reduce of a wavefront's rows by group key, the
global open-addressing table probe (``csrc/kernels/hash_agg.hip`` layout), and the run top-K
walk (per-lane top-2 registers, the cross-window carry, the per-wavefront slot flush) of
``exec/hash_agg.py TopKPlan``.  Emitters return lines of HIP source; variables follow the
generators' ``x<slot>`` / ``n<slot>`` naming (callers rename)."""
from __future__ import annotations

import re
from typing import List

from ..ops import _lib as NL
from . import jit as J


HASH_MAX_PROBE = 512


def _hash_key_lines(gen: J._Gen, hk, var: str, sfx: str, ind: str) -> List[str]:
    """``u64 <var>`` = the packed / raw hash key from the key columns ``x<slot><sfx>``, and
    ``bool <var>_nul``."""
    a = gen.a
    b = []
    if hk.mode == "packed":
        b.append(f"{ind}u64 {var} = 0ull; const bool {var}_nul = false;")
        for j, c in enumerate(hk.cols):
            lo = a.add("q", f"HL{j}", "long long")
            sh = a.add("q", f"HS{j}", "long long")
            s = c.slot
            x = f"x{s}{sfx}"
            if c.kind == "f32":
                val = f"hs_f32key((float){x})"
            elif c.kind == "dec":
                sc = a.add("d", f"HQ{j}", "double")
                val = f"(u64)((i64)__builtin_rint((double){x} * {sc}) - {lo})"
            else:
                val = f"(u64)((i64){x} - {lo})"
            ok = gen.ok(s)
            if sfx:
                ok = re.sub(rf"\bn{s}\b", f"n{s}{sfx}", ok)
            expr = f"({ok} ? {val} + 1ull : 0ull)" if c.nullable else val
            b.append(f"{ind}{var} |= {expr} << (unsigned){sh};")
    else:
        c = hk.cols[0]
        s = c.slot
        x = f"x{s}{sfx}"
        val = f"hs_f64key((double){x})" if hk.mode == "raw_float" else f"(u64)(i64){x}"
        ok = gen.ok(s)
        if sfx:
            ok = re.sub(rf"\bn{s}\b", f"n{s}{sfx}", ok)
        nul = f"!{ok}" if c.nullable else "false"
        b.append(f"{ind}const bool {var}_nul = {nul}; const u64 {var} = {var}_nul ? 0ull : {val};")
    return b


def _hash_accumulate(gen: J._Gen, aggs, hk, pass_var: str, ind: str, tk=None,
                     seg: str = None, row: str = None, run: str = None,
                     carry_gen: "J._Gen" = None) -> List[str]:
    """Hash-mode grouping (``hk``: an exec.hash_agg.KeyPlan): the wavefront's lanes, in row
    order, are cut into runs of equal group keys (one ballot of the run heads); a segmented
    shuffle scan sums each run's values into its last lane, and only that lane probes the
    global table (linear probing, 64-bit key, atomicCAS insert) and adds the run's partials
    with memory-side atomics.  Inputs sorted by a key prefix (index scans, merge-join output)
    put a group's rows in adjacent lanes, so most groups cost one probe and one atomic per
    aggregate per 64-row batch.  Variables are ``x<slot>`` / ``n<slot>`` (callers rename).

    ``seg``: a per-lane variable that identifies the group within the batch (the key run of
    the key-run walk): lanes are cut on it, and the key columns are loaded (``_uload``) only
    by lanes that emit a group (a table probe or a top-K candidate), not for every row.
    ``tk``: the run top-K walk instead (``_topk_accumulate``)."""
    if tk is not None:
        return _topk_accumulate(gen, aggs, hk, pass_var, ind, tk, seg, row, run, carry_gen)
    i2 = ind + "  "
    b = [f"{ind}{{ const int hln = (int)(threadIdx.x & 63u); const bool hok = {pass_var};"]
    if seg is None:
        b.extend(_hash_key_lines(gen, hk, "hk", "", i2))
        b.append(f"{i2}const bool hnul = hk_nul;")
        b += [f"{i2}const u64 hkp = __shfl_up(hk, 1u, 64);",
              f"{i2}const int hfp = __shfl_up((hok ? 1 : 0) | (hnul ? 2 : 0), 1u, 64);",
              f"{i2}const bool hsame = hln > 0 && hok && (hfp & 1) != 0 && "
              f"((hfp >> 1) & 1) == (hnul ? 1 : 0) && hkp == hk;"]
    else:
        b += _seg_heads(seg, i2)
    b += [f"{i2}const u64 hH = __ballot(!hsame);",
          f"{i2}const int hss = 63 - __builtin_clzll(hH & ((2ull << hln) - 1ull));",
          f"{i2}const bool htl = hok && (hln == 63 || ((hH >> ((hln + 1) & 63)) & 1ull) != 0ull);"]
    b += _seg_reduce(gen, aggs, hk, i2)
    if seg is not None:
        _lazy_key(gen, hk, "htl", b, i2)
    b += _hash_probe(gen, aggs, hk, "htl", i2, "hk", "hnul", "hv{i}", "hc{i}",
                     "(unsigned long long)(hln - hss + 1)")
    b.append(f"{ind}}}")
    return b


def _seg_heads(seg: str, ind: str) -> List[str]:
    return [f"{ind}const unsigned hsg = (unsigned){seg};",
            f"{ind}const unsigned hsp = __shfl_up(hsg, 1u, 64);",
            f"{ind}const int hfp = __shfl_up(hok ? 1 : 0, 1u, 64);",
            f"{ind}const bool hsame = hln > 0 && hok && hfp != 0 && hsp == hsg;"]


def _seg_reduce(gen: J._Gen, aggs, hk, ind: str) -> List[str]:
    """Per lane ``hv<i>`` (value) / ``hc<i>`` (own non-null count) summed over its segment's
    lanes up to it (segmented shuffle scan: a segment's tail lane holds the segment's total)."""
    own = hk.own_counts
    b, red = [], []
    for i, ag in enumerate(aggs):
        if ag.kind == NL.AK_COUNT_STAR:
            continue
        v, ok = gen.agg_value(i, ag)
        b.append(f"{ind}const bool hq{i} = hok && {ok};")
        if ag.kind != NL.AK_COUNT:
            b.append(f"{ind}double hv{i} = hq{i} ? (double)({v}) : {J._ident(ag.kind)};")
            op = "fmin" if ag.kind == NL.AK_MIN else ("fmax" if ag.kind == NL.AK_MAX else None)
            red.append((f"hv{i}", "double", op))
        if own[i]:
            b.append(f"{ind}long long hc{i} = hq{i} ? 1ll : 0ll;")
            red.append((f"hc{i}", "long long", None))
    if red:
        b.append(f"{ind}#pragma unroll")
        b.append(f"{ind}for (int hd = 1; hd < 64; hd <<= 1) {{")
        for var, ct, _ in red:
            b.append(f"{ind}  const {ct} u_{var} = __shfl_up({var}, (unsigned)hd, 64);")
        b.append(f"{ind}  if (hln - hd >= hss) {{")
        for var, _, op in red:
            b.append(f"{ind}    {var} = " + (f"{op}({var}, u_{var});" if op else f"{var} + u_{var};"))
        b.append(f"{ind}  }}")
        b.append(f"{ind}}}")
    return b


def _lazy_key(gen: J._Gen, hk, cond: str, out: List[str], ind: str, key: str = "hk",
              nul: str = "hnul") -> None:
    """``key`` / ``nul`` of lanes where ``cond`` holds, from the key columns loaded there (at
    ``gen``'s row)."""
    out.append(f"{ind}u64 {key} = 0ull; bool {nul} = false;")
    out.append(f"{ind}if ({cond}) {{")
    for c in hk.cols:
        J._uload(gen, c.slot, "KK", out, ind + "  ")
    out.extend(_hash_key_lines(gen, hk, "hk_l", "_KK", ind + "  "))
    out.append(f"{ind}  {key} = hk_l; {nul} = hk_l_nul; }}")


def _hash_probe(gen: J._Gen, aggs, hk, cond: str, ind: str, key: str, nul: str, sv: str, cv: str,
                rn: str) -> List[str]:
    """Lanes where ``cond`` holds add one group's partials to the global table: sums ``sv``,
    own counts ``cv`` (templates over the aggregate index ``{i}``), ``rn`` rows.  CAS-first
    probe: a group's first insert is one returning atomic (no load first); later inserts of
    the same group find it on the first CAS of their probe."""
    a = gen.a
    kp = a.add("p", "hkeys", "unsigned long long*")
    sp = a.add("p", "hsum", "double*")
    cp = a.add("p", "hcnt", "long long*")
    mm = any(x.kind in (NL.AK_MIN, NL.AK_MAX) for x in aggs)
    mnp = a.add("p", "hmin", "double*") if mm else None
    mxp = a.add("p", "hmax", "double*") if mm else None
    hm = a.add("q", "HM", "long long")
    fl = a.add("p", "hflag", "long long*")
    own = hk.own_counts
    b = [f"{ind}if ({cond}) {{",
         f"{ind}  long long hs_ = -1;",
         f"{ind}  if ({nul}) hs_ = {hm} + 1; else if ({key} == ~0ull) hs_ = {hm}; else {{",
         f"{ind}    u64 hh = hs_mix64({key}) & (u64)({hm} - 1);",
         f"{ind}    for (int pr_ = 0; pr_ < {HASH_MAX_PROBE}; ++pr_) {{",
         f"{ind}      const u64 pv_ = atomicCAS(&{kp}[hh], ~0ull, {key});",
         f"{ind}      if (pv_ == ~0ull || pv_ == {key}) {{ hs_ = (long long)hh; break; }}",
         f"{ind}      hh = (hh + 1ull) & (u64)({hm} - 1);",
         f"{ind}    }}",
         f"{ind}    if (hs_ < 0) {fl}[0] = 1;",
         f"{ind}  }}",
         f"{ind}  if (hs_ >= 0) {{",
         f"{ind}    const long long hst = {hm} + 2;   // SoA: aggregate i of slot s at i * (M + 2) + s",
         f"{ind}    const unsigned long long hrn = {rn};"]
    for i, ag in enumerate(aggs):
        cnt = f"(unsigned long long)({cv.format(i=i)})" if own[i] else "hrn"
        tgt = f"(unsigned long long*)&{cp}[{i} * hst + hs_]"
        if ag.kind == NL.AK_COUNT_STAR:
            # the implicit COUNT(*) is kept only when a result needs it (COUNT / AVG); group
            # occupancy is the key word, except for the two direct slots
            if hk.need_star:
                b.append(f"{ind}    atomicAdd({tgt}, {cnt});")
            else:
                b.append(f"{ind}    if (hs_ >= {hm}) atomicAdd({tgt}, {cnt});")
            continue
        if ag.kind == NL.AK_COUNT:
            b.append(f"{ind}    atomicAdd({tgt}, {cnt});")
            continue
        v = sv.format(i=i)
        if ag.kind == NL.AK_SUM:
            b.append(f"{ind}    unsafeAtomicAdd(&{sp}[{i} * hst + hs_], {v});")
        elif ag.kind == NL.AK_MIN:
            b.append(f"{ind}    atomicMin(&{mnp}[{i} * hst + hs_], {v});")
        else:
            b.append(f"{ind}    atomicMax(&{mxp}[{i} * hst + hs_], {v});")
        if own[i]:
            b.append(f"{ind}    atomicAdd({tgt}, {cnt});")
    b += [f"{ind}  }}", f"{ind}}}"]
    return b


def _topk_accumulate(gen: J._Gen, aggs, hk, pass_var: str, ind: str, tk, seg: str, row: str,
                     run: str, carry_gen: "J._Gen") -> List[str]:
    """Run top-K walk (hash_agg.TopKPlan) over one 64-entry window of the key-run walk's list
    (entries in row order, a prefix of the lanes valid; ``seg`` the entry's key run in the
    window, ``run`` its absolute run index, ``row`` its row).  A key's passing rows are one
    contiguous stretch of the wavefront's entries, so segments are completed across windows
    by a carry: the window's last segment is carried (sums, counts, rows, a row of the key,
    kernel-scope ``tc*`` registers) into the next window, whose first segment adds it when it
    continues the same run; otherwise the carry is complete and emitted by lane 0.  Complete
    segments go to the lanes' top-2 registers (``_topk_insert``); the table takes only
    segments that may continue outside the wavefront's tiles: one that starts the
    wavefront's walk (``tco_``, it may have rows in the previous wavefront's tiles) and the
    final carry (``_topk_carry_final``)."""
    i2 = ind + "  "
    i3 = i2 + "  "
    own = hk.own_counts
    b = [f"{ind}{{ const int hln = (int)(threadIdx.x & 63u); const bool hok = {pass_var};",
         f"{i2}const u64 hV_ = __ballot(hok);",
         f"{i2}if (hV_ != 0ull) {{"]
    b += _seg_heads(seg, i3)
    b += [f"{i3}const u64 hH = __ballot(!hsame);",
          f"{i3}const int hss = 63 - __builtin_clzll(hH & ((2ull << hln) - 1ull));",
          f"{i3}const bool htl = hok && (hln == 63 || ((hH >> ((hln + 1) & 63)) & 1ull) != 0ull);",
          f"{i3}const int hlast_ = 63 - __builtin_clzll(hV_);",
          f"{i3}const long long hrun_ = hok ? (long long)({run}) : -1ll;",
          f"{i3}const long long hr0_ = __shfl(hrun_, 0, 64);",
          # the first segment continues the carried one / starts the wavefront's walk
          f"{i3}const bool hmg_ = tcr_ == hr0_;",
          f"{i3}const bool hol_ = hmg_ ? tco_ : (tcr_ < 0);"]
    b += _seg_reduce(gen, aggs, hk, i3)
    b.append(f"{i3}long long hrn_ = (long long)(hln - hss + 1);")
    merge = [f" hrn_ += tcn_;"]
    for i, ag in enumerate(aggs):
        if ag.kind not in (NL.AK_COUNT_STAR, NL.AK_COUNT):
            merge.append(f" hv{i} += tcv{i};")
        if own[i]:
            merge.append(f" hc{i} += tcc{i};")
    b.append(f"{i3}if (hmg_ && hss == 0) {{" + "".join(merge) + " }")
    b += [f"{i3}const bool hopen_ = hss == 0 && hol_;",
          f"{i3}const bool hlst_ = htl && hln == hlast_;",
          f"{i3}const bool hcomp = htl && !hlst_ && !hopen_;",
          f"{i3}const bool hprb_ = htl && !hlst_ && hopen_;"]
    b += _topk_value(aggs, hk, tk, i3, "hv{i}", "hc{i}", "hrn_", "tkv_")
    _lazy_key(gen, hk, "hprb_", b, i3)
    b += _hash_probe(gen, aggs, hk, "hprb_", i3, "hk", "hnul", "hv{i}", "hc{i}",
                     "(unsigned long long)hrn_")
    b += _topk_insert(aggs, hk, tk, i3, row, "hcomp", "hv{i}", "hc{i}", "hrn_", "tkv_")
    # the carry, complete when this window does not continue it: lane 0 emits it
    b.append(f"{i3}if (tcr_ >= 0 && !hmg_) {{")
    b += _topk_carry_emit(aggs, hk, tk, i3 + "  ", carry_gen)
    b.append(f"{i3}}}")
    # the window's last segment becomes the carry
    b += [f"{i3}tcr_ = __shfl(hrun_, hlast_, 64);",
          f"{i3}tco_ = __shfl(hopen_ ? 1 : 0, hlast_, 64) != 0;",
          f"{i3}tcw_ = __shfl((long long)({row}), hlast_, 64);",
          f"{i3}tcn_ = __shfl(hrn_, hlast_, 64);"]
    for i, ag in enumerate(aggs):
        if ag.kind not in (NL.AK_COUNT_STAR, NL.AK_COUNT):
            b.append(f"{i3}tcv{i} = __shfl(hv{i}, hlast_, 64);")
        if own[i]:
            b.append(f"{i3}tcc{i} = __shfl(hc{i}, hlast_, 64);")
    b += [f"{i2}}}", f"{ind}}}"]
    return b


def _topk_carry_emit(aggs, hk, tk, ind: str, carry_gen: "J._Gen") -> List[str]:
    """Lane 0 emits the carried segment (complete): to its top-2 registers, or to the table
    when the segment may have rows before the wavefront's walk (``tco_``)."""
    b = [f"{ind}const bool hce_ = hln == 0;",
         f"{ind}const bool hct_ = hce_ && !tco_;",
         f"{ind}const bool hcp_ = hce_ && tco_;"]
    b += _topk_value(aggs, hk, tk, ind, "tcv{i}", "tcc{i}", "tcn_", "tcv_")
    _lazy_key(carry_gen, hk, "hcp_", b, ind, "hck_", "hcn_")
    b += _hash_probe(carry_gen, aggs, hk, "hcp_", ind, "hck_", "hcn_", "tcv{i}", "tcc{i}",
                     "(unsigned long long)tcn_")
    b += _topk_insert(aggs, hk, tk, ind, "tcw_", "hct_", "tcv{i}", "tcc{i}", "tcn_", "tcv_")
    return b


def _topk_carry_final(aggs, hk, tk, ind: str, carry_gen: "J._Gen") -> List[str]:
    """After the walk: the last carry may continue in the next wavefront's tiles - lane 0 adds
    it to the table."""
    b = [f"{ind}if (tcr_ >= 0) {{",
         f"{ind}  const int hln = (int)(threadIdx.x & 63u);",
         f"{ind}  const bool hcp_ = hln == 0;"]
    _lazy_key(carry_gen, hk, "hcp_", b, ind + "  ", "hck_", "hcn_")
    b += _hash_probe(carry_gen, aggs, hk, "hcp_", ind + "  ", "hck_", "hcn_", "tcv{i}",
                     "tcc{i}", "(unsigned long long)tcn_")
    b.append(f"{ind}}}")
    return b


def _topk_values(aggs, hk, sv: str = "hv{i}", cv: str = "hc{i}", rn: str = "hrn_"):
    """Per aggregate i: (sum expression, count expression) a complete segment stores, matching
    what the hash table would hold for that group (counts only where the table keeps them)."""
    own = hk.own_counts
    out = []
    for i, ag in enumerate(aggs):
        if ag.kind == NL.AK_COUNT_STAR:
            out.append(("0.0", rn if hk.need_star else "0ll"))
        elif ag.kind == NL.AK_COUNT:
            out.append(("0.0", cv.format(i=i) if own[i] else rn))
        else:
            out.append((sv.format(i=i), cv.format(i=i) if own[i] else "0ll"))
    return out


def _topk_value(aggs, hk, tk, ind: str, sv: str = "hv{i}", cv: str = "hc{i}",
                rn: str = "hrn_", out: str = "tkv_") -> List[str]:
    """``out``: a segment's order value in the "larger is better" image."""
    s, c = _topk_values(aggs, hk, sv, cv, rn)[tk.agg]
    ov = f"(double)({c})" if tk.src_count else s
    sign = "" if tk.desc else "-"
    return [f"{ind}const double {out} = {sign}({ov});"]


TOPK_LANE = 2   # entries each lane keeps (hash_agg.TopKPlan)


def _topk_decls(aggs, tk) -> List[str]:
    """Kernel-scope state of the run top-K (hash_agg.TopKPlan): each lane keeps its best
    ``TOPK_LANE`` complete segments in registers (entry 0 the better; the tail row, whose key
    is read only at the end, the order value and the aggregates) and ``tkdmx``, the largest
    value it dropped; and the wavefront's carried segment (``_topk_accumulate``): its
    absolute run (-1: none yet), whether it may start before the walk, a row of its key, its
    rows and per-aggregate sums / counts."""
    b = ["  double tkdmx = -__builtin_inf();",
         "  long long tcr_ = -1, tcw_ = 0, tcn_ = 0; bool tco_ = false;"]
    b.append("  " + " ".join(f"double tcv{i} = 0.0; long long tcc{i} = 0ll;"
                             for i in range(len(aggs))))
    for j in range(TOPK_LANE):
        b.append(f"  i64 tkr{j} = -1; double tkv{j} = -__builtin_inf();" +
                 "".join(f" double tks{j}_{i} = 0.0; long long tkc{j}_{i} = 0ll;"
                         for i in range(len(aggs))))
    return b


def _topk_insert(aggs, hk, tk, ind: str, row: str, cond: str = "hcomp", sv: str = "hv{i}",
                 cv: str = "hc{i}", rn: str = "hrn_", val: str = "tkv_") -> List[str]:
    """A complete segment's lane keeps it if it beats the lane's worse entry (a lane-local
    insertion into a sorted pair: no cross-lane work and no memory traffic per key); anything
    displaced or not kept raises the lane's dropped maximum."""
    assert TOPK_LANE == 2    # the shift-or-set insertion below is exact for a pair
    vals = _topk_values(aggs, hk, sv, cv, rn)

    def put(j):
        return f" tkr{j} = {row}; tkv{j} = {val};" + "".join(
            f" tks{j}_{i} = (double)({sx}); tkc{j}_{i} = (long long)({cx});"
            for i, (sx, cx) in enumerate(vals))
    mv = " tkr1 = tkr0; tkv1 = tkv0;" + "".join(
        f" tks1_{i} = tks0_{i}; tkc1_{i} = tkc0_{i};" for i in range(len(vals)))
    return [f"{ind}if ({cond}) {{",
            f"{ind}  if ({val} > tkv1) {{",
            f"{ind}    tkdmx = fmax(tkdmx, tkv1);",
            f"{ind}    if ({val} > tkv0) {{{mv}{put(0)} }} else {{{put(1)} }}",
            f"{ind}  }} else {{ tkdmx = fmax(tkdmx, {val}); }}",
            f"{ind}}}"]


def _topk_flush(aggs, tk, args: "Args", wid: str, key_lines) -> List[str]:
    """The wavefront's best K entries to its K slots of the candidate arrays (keys, order-value
    images - unsigned, smallest first, as hs_topk_select reads them - then per aggregate sums /
    counts at stride TKCAP; empty slots: key ~0, image of -inf), its K-th best value (TKW,
    signed image) and its dropped maximum (TKD) - found by a bitwise search
    over the lanes' order-preserving images (64 ballots), no atomics.  ``key_lines(j, ind)``
    loads entry j's key into ``tkey_`` from its row."""
    K = tk.K
    kk = args.add("p", "TKK", "unsigned long long*")
    kv = args.add("p", "TKV", "long long*")
    ks = args.add("p", "TKS", "double*")
    kc = args.add("p", "TKC", "long long*")
    kw = args.add("p", "TKW", "long long*")
    kd = args.add("p", "TKD", "long long*")
    cap = args.add("q", "TKCAP", "long long")
    imgs = " + ".join(f"__popcll(__ballot(tki{j} >= t_))" for j in range(TOPK_LANE))
    b = ["  { const int tl_ = (int)(threadIdx.x & 63u);",
         "    " + " ".join(f"const u64 tki{j} = (u64)hs_dimg(tkv{j}) ^ 0x8000000000000000ull;"
                           for j in range(TOPK_LANE)),
         "    u64 th_ = 0ull;",
         "    for (int b_ = 63; b_ >= 0; --b_) { const u64 t_ = th_ | (1ull << b_);",
         f"      if ({imgs} >= {K}) th_ = t_; }}",
         "    // th_: the K-th best image (0 when fewer than K entries are live)",
         "    double dm_ = tkdmx;",
         "    long long pos_ = 0;"]
    for j in range(TOPK_LANE):
        b += [f"    {{ const bool lv_ = tkr{j} >= 0 && tki{j} >= th_;",
              "      const u64 lb_ = __ballot(lv_);",
              "      const long long at_ = pos_ + __popcll(lb_ & ((1ull << tl_) - 1ull));",
              f"      if (lv_ && at_ < {K}) {{",
              f"        const long long te_ = (long long)({wid}) * {K} + at_;"]
        b += key_lines(j, "        ")
        b += [f"        {kk}[te_] = tkey_; {kv}[te_] = (long long)~tki{j};"]
        for i in range(len(aggs)):
            b.append(f"        {ks}[{i} * {cap} + te_] = tks{j}_{i}; "
                     f"{kc}[{i} * {cap} + te_] = tkc{j}_{i};")
        b += [f"      }} else if (tkr{j} >= 0) dm_ = fmax(dm_, tkv{j});",
              "      pos_ += __popcll(lb_); }"]
    b += [f"    for (long long e_ = pos_ + tl_; e_ < {K}; e_ += 64) {{",
          f"      const long long te_ = (long long)({wid}) * {K} + e_;",
          f"      {kk}[te_] = ~0ull; {kv}[te_] = (long long)~((u64)hs_dimg(-__builtin_inf()) ^ "
          "0x8000000000000000ull); }",
          "    for (int o_ = 32; o_ > 0; o_ >>= 1) dm_ = fmax(dm_, __shfl_xor(dm_, o_, 64));",
          "    if (tl_ == 0) {",
          f"      {kw}[{wid}] = pos_ >= {K} ? (long long)(th_ ^ 0x8000000000000000ull) : "
          "hs_dimg(-__builtin_inf());",
          f"      {kd}[{wid}] = hs_dimg(dm_); }}",
          "  }"]
    return b
