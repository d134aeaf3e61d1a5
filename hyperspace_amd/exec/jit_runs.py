"""Two-phase run-keyed merge join + aggregate (the MI355X form of a co-located bucketed
SortMergeJoin whose right key is unique: JoinIndexRule.scala:63-69).

The left key is in its run-length form (exec/encoding.RunCompact: per 64-row group a run-start
mask ``gmask`` and the first row's run ``gruns``, plus one key per run ``runkeys``).  Instead of
one kernel that stages, matches and aggregates per tile, the join is split by what each phase
streams:

1. ``hs_jit_run_tags`` - per merge-join tile, the tile's right key span is staged in LDS with
   the right side's predicates evaluated once per right row; each thread matches a contiguous
   chunk of the tile's runs (one LDS binary search, then a walk) and writes a W-bit **tag** per
   run into a bitmap: 0 = no (passing) right row, else 1 (ungrouped / left-grouped) or the
   right-side group code + 1.  Tags are assembled in LDS and leave as whole 32-bit words (only
   a tile's two edge words use an atomic OR).  It reads the run keys, the right keys and the
   right predicate columns once: ~1.5 GB at TPC-H SF100.
2. ``hs_jit_run_scan`` - a streaming scan of the left rows (vector loads, no LDS staging, no
   barriers): row -> run index from the group mask by one popcount, tag from the bitmap (the
   NI rows of a thread touch one or a few adjacent words), left predicates, and the compacted
   aggregate tail over the passing rows only.

Both phases are plain streams, so each runs near the HBM roofline; the single-kernel form
(jit.gen_merge_join_agg) keeps a long chain of dependent round trips per tile.  The two-phase
form applies when no aggregate input comes from the right side, every right predicate reads
only right columns, and a right-side group key (if any) has at most 255 groups."""
from __future__ import annotations

from typing import List, Optional

from ..ops import _lib as NL
from . import jit as J
from . import jit_hash as JH

SPLIT = 8
# tunables: fields of exec.kernel_config.KernelConfig (bound by kernel_config.bind)
from . import kernel_config as _KC  # noqa: E402
_CFG = _KC.active()
MJ_2P, RS_ITEMS = _CFG.mj_2p, _CFG.rs_items
RT2_UNROLL, RT2_GRID, RT2_I32 = _CFG.rt2_unroll, _CFG.rt2_grid, _CFG.rt2_i32
RT2_MATCH, RT2_COPY, RT2_LO16 = _CFG.rt2_match, _CFG.rt2_copy, _CFG.rt2_lo16
RS_BITS, RS_BITS_GRID, RS_PACK = _CFG.rs_bits, _CFG.rs_bits_grid, _CFG.rs_pack
RS_PIPE, RS_WALK, RS_LDS, RS_LUT = _CFG.rs_pipe, _CFG.rs_walk, _CFG.rs_lds, _CFG.rs_lut
RS_PK16, RS_WAVES, RS_PACK12 = _CFG.rs_pk16, _CFG.rs_waves, _CFG.rs_pack12


def tag_width(p: NL.JoinParams) -> int:
    """Bits per run tag, or 0 when the two-phase form does not apply to ``p``."""
    if p.group_col >= SPLIT:
        if p.num_groups > 255:
            return 0
        for w in (1, 2, 4, 8):
            if p.num_groups + 1 <= (1 << w):
                return w
    return 1


def applies(p: NL.JoinParams) -> bool:
    if not MJ_2P:
        return False
    for i in range(p.naggs):
        a = p.aggs[i]
        if any(a.col[t] >= SPLIT for t in range(a.nterms)) and a.kind != NL.AK_COUNT_STAR:
            return False
    if not J._right_only(p, SPLIT):
        return False
    if p.group_col >= SPLIT and p.cols[p.group_col].valid:
        return False
    return tag_width(p) > 0


def _rpreds(p):
    return [(k, p.preds[k]) for k in range(p.nlp, p.npreds)]


def _lpreds(p):
    return [(k, p.preds[k]) for k in range(p.nlp)]


# phase 1: 64-run groups per unrolled iteration of a wavefront (gen_run_tags2)


def tags2_shape(p: NL.JoinParams, compacts, W: int, ix32: bool = False, mode: str = "") -> tuple:
    cols = tuple(sorted((s, c) for s, c in J._col_specs(p, compacts).items()
                        if s >= SPLIT or s == p.lkey))
    preds = tuple((p.preds[k].kind, p.preds[k].op, p.preds[k].col, p.preds[k].col2,
                   p.preds[k].group) for k in range(p.nlp, p.npreds))
    return ("run_tags2", cols, preds, p.nlp, p.lkey, p.rkey, _tags_grouped(p) and p.group_col,
            W, RT2_UNROLL, J.BLOCK, ix32, mode)


def _stage_slots(p: NL.JoinParams) -> list:
    """Right columns phase 1 reads at a matched row: predicate columns and the group key."""
    return list(dict.fromkeys(J._pred_slots(_rpreds(p)) +
                              ([p.group_col] if _tags_grouped(p) else [])))


def _tags_grouped(p: NL.JoinParams) -> bool:
    """Whether the tags carry a right-side group code: a right group key with more than one
    group (a single group's domain [group_base, group_base + 1) holds every value of the column,
    which is non-null here: ``applies``)."""
    return p.group_col >= SPLIT and p.num_groups > 1


def gen_run_tags2(p: NL.JoinParams, compacts, W: int, ix32: bool = False,
                  mode: str = "") -> J.Kernel:
    """Phase 1, direct form: no tiles and no LDS.  Each wavefront owns a contiguous chunk of
    64-run groups of the left run list (so it owns whole 2W-word stretches of the tag bitmap
    and stores them without atomics).  Lane l of a group guesses the right row of its run: the
    previous group's last match + 1 + l (or, at a range start, the range-relative position) -
    exact for a foreign key whose every right key has left rows, the common case - and verifies
    it with one compare of the 32-bit key images; a mismatch gallops from the guess to the
    lower bound (exact for any sorted unique right keys).  The right predicate and group
    columns are loaded at the guess together with the key, so a verified guess costs one round
    trip; RT2_UNROLL groups are in flight per iteration.

    Ranges (``RNG``, NRG x 4 int64, sorted by first run): [first run, end run) of each left row
    range and the right bucket's rows [s0, s1).  (16-bit grouped run keys measured 0.59 vs
    0.29 ms - more dependent loads per run - and a per-tile LDS form 0.79 ms: both removed.)

    ``ix32``: run and right-row indices fit int32 (the lowering checks the table sizes), so the
    index arithmetic, range clamps and gallop run in 32-bit registers and the column loads
    address through a scalar base plus a 32-bit lane offset - the 64-bit index math was most of
    the kernel's VALU instructions (``profiles/pmc_query_kernels_sf100_r6.txt``).

    ``mode``: "rec" also stores each run's matched right row (or -1) into ``MOUT``; "match"
    reads that record (``MATCH``, one int32 per run, -1 padded to whole 64-run groups) instead of
    the left run keys, the right key images and the range table - it depends only on the
    lowering's ranges and the key columns, not on the literals (``record_matches``)."""
    IX = "int" if ix32 else "i64"  # noqa: N806 — run / right-row index type
    args = J.Args()
    if mode in ("match", "copy"):
        return _gen_tags2_match(p, compacts, W, mode == "copy")
    lk, rk = p.lkey, p.rkey
    args.add("p", f"RK{lk}", "const int*")
    args.add("p", "RNG", "const long long*")
    args.add("p", "tags", "unsigned*")
    for n in ("NRG", "NRUNS", "KLO", "KSP", "KOF"):
        args.add("q", n, "long long")
    cols = J._col_specs(p, compacts)
    rpreds = _rpreds(p)
    rgroup = _tags_grouped(p)
    stage_slots = _stage_slots(p)
    U = max(1, RT2_UNROLL)  # noqa: N806
    WV = J.BLOCK // 64  # noqa: N806
    MASK = (1 << W) - 1  # noqa: N806
    if mode == "rec":
        assert ix32
        args.add("p", "MOUT", "int*")
    lo16 = mode in ("lo16", "lo16prep")
    if lo16:
        assert ix32
        cst = "" if mode == "lo16prep" else "const "
        args.add("p", "LL", f"{cst}unsigned short*")
        args.add("p", "RL", f"{cst}unsigned short*")
    g = J._Gen(args, cols, SPLIT, ("row_", "row_"), frozenset(), True)
    rv = J._valid_expr(g, rk, "row_")
    if rgroup:
        gb = args.add("q", "group_base", "long long")
        ng = args.add("q", "num_groups", "long long")
    renc = cols[rk][2]
    if renc and len(renc) > 2 and renc[2] == 64:
        # grouped 16-bit right key: code = gbase[row >> 6] + offset, or the 32-bit code of a
        # wide group (both loads unconditional: the wide one hits row 0 otherwise)
        assert rk not in stage_slots
        base = args.add("q", f"B{rk}", "long long")
        gp = args.add("p", f"G{rk}", "const int*")
        wp = args.add("p", f"W{rk}", "const int*")
        cp = g.ptr(rk)
        rval = (f"({{ const int gb_ = {gp}[row_ >> 6]; const bool wd_ = gb_ == (int)0x80000000; "
                f"const int w_ = {wp}[wd_ ? row_ : 0]; const unsigned short o_ = {cp}[row_]; "
                f"{base} + (wd_ ? (i64)w_ : (i64)gb_ + (i64)o_); }})")
        # the guess's image without the dependent wide-group load: 0 (below every left image,
        # so never a false match) for a wide group; a miss re-reads the exact image
        fval = (f"({{ const int gb_ = {gp}[row_ >> 6]; const unsigned short o_ = {cp}[row_]; "
                f"gb_ == (int)0x80000000 ? (i64)-1 : {base} + (i64)gb_ + (i64)o_; }})")
    else:
        rval = fval = g.value(rk, "row_")

    def image(val: str, wide0: bool) -> str:
        guard = "(__v_ == (i64)-1) || " if wide0 else ""
        return (f"({rv} ? 0u : ({{ const i64 __v_ = (i64)({val}); const i64 d_ = __v_ - a.KLO; "
                f"({guard}d_ < 0) ? 0u : (d_ > a.KSP ? 0xFFFFFFFFu : (unsigned)(d_ + 1)); }}))")
    img = image(rval, False)
    imgf = image(fval, fval is not rval)

    def tag_expr(gen: J._Gen, it, ok: str) -> str:
        cond = J._rename(gen.cnf(rpreds), stage_slots, it)
        if not rgroup:
            return f"(({ok}) && {cond} ? 1u : 0u)"
        gx = J._rename(f"x{p.group_col}", stage_slots, it)
        return (f"({{ const i64 gl_ = (i64){gx} - {gb}; (({ok}) && {cond} && gl_ >= 0 && "
                f"gl_ < {ng}) ? (unsigned)(gl_ + 1) : 0u; }})")

    if mode == "lo16prep":
        # the low 16 bits of every left run key image and right key image (``lo16_keys``)
        args.add("q", "NRIGHT", "long long")
        body = [f"  auto IMG = [&]({IX} row_) -> unsigned {{ return {img}; }};",
                f"  const i64 t_ = (i64)blockIdx.x * {J.BLOCK} + threadIdx.x, "
                f"n_ = (i64)gridDim.x * {J.BLOCK};",
                f"  for (i64 i = t_; i < a.NRUNS; i += n_) "
                f"a.LL[i] = (unsigned short)((unsigned)a.RK{lk}[i] + (unsigned)a.KOF);",
                "  for (i64 i = t_; i < a.NRIGHT; i += n_) a.RL[i] = (unsigned short)IMG((int)i);"]
        src = (J._PRELUDE + args.struct_src() +
               f'extern "C" __global__ __launch_bounds__({J.BLOCK}) void hs_jit_key_lo16(Args a) '
               "{\n" + "\n".join(body) + "\n}\n")
        return J.Kernel(src, "hs_jit_key_lo16", args)

    b: List[str] = [
        f"  auto IMG = [&]({IX} row_) -> unsigned {{ return {img}; }};",
        f"  auto IMGF = [&]({IX} row_) -> unsigned {{ return {imgf}; }};",
        "  const int lane = (int)(threadIdx.x & 63);",
        "  const i64 G = (a.NRUNS + 63) >> 6;",
        f"  const i64 nwv = (i64)gridDim.x * {WV};",
        # wavefront-uniform (scalar registers, scalar loads of the range table)
        f"  const i64 wv = (i64)blockIdx.x * {WV} + "
        "(i64)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));",
        "  const i64 per = (G + nwv - 1) / nwv;",
        "  const i64 gbeg = wv * per;",
        "  const i64 gend = G < gbeg + per ? G : gbeg + per;",
        "  if (gbeg >= gend || a.NRG <= 0) return;",
        "  const i64* RG = a.RNG;",
        "  int rg = 0;",
        "  { int lo = 0, hi = (int)a.NRG; const i64 r0 = gbeg << 6;",
        "    while (hi - lo > 1) { const int m = (lo + hi) >> 1; "
        "if (RG[4 * m] <= r0) lo = m; else hi = m; }",
        "    rg = lo; }",
        f"  {IX} lr0 = ({IX})RG[4 * rg], lr1 = ({IX})RG[4 * rg + 1], s0 = ({IX})RG[4 * rg + 2], "
        f"s1 = ({IX})RG[4 * rg + 3];",
        "  i64 nxt0 = rg + 1 < a.NRG ? RG[4 * (rg + 1)] : 0x7fffffffffffffffll;",
        f"  {IX} gbase = -1;   // right row of the next group's first run (-1: range-relative)",
        f"  for (i64 gi = gbeg; gi < gend; gi += {U}) {{",
        "    while (nxt0 <= (gi << 6)) {",
        f"      ++rg; lr0 = ({IX})RG[4 * rg]; lr1 = ({IX})RG[4 * rg + 1]; s0 = ({IX})RG[4 * rg + 2];",
        f"      s1 = ({IX})RG[4 * rg + 3]; gbase = -1;",
        "      nxt0 = rg + 1 < a.NRG ? RG[4 * (rg + 1)] : 0x7fffffffffffffffll; }",
        # wavefront-uniform: every run of this iteration's groups belongs to range rg (or none)
        f"    if (((gi + {U}) << 6) <= nxt0) {{"]
    ind = "      "

    def group(u: int, fast: bool, ind: str) -> None:
        """Loads and guess of group u: unconditional (clamped) loads in the fast form, so all
        U groups' loads are in flight together (a load under a per-lane condition makes the
        compiler wait for it before the branches merge)."""
        b.extend([f"{ind}const {IX} r{u} = ({IX})(((gi + {u}) << 6) + lane);",
                  f"{ind}const bool in{u} = gi + {u} < gend;"])
        if fast:
            b.append(f"{ind}const {IX} l0_{u} = lr0, l1_{u} = lr1, a0_{u} = s0, a1_{u} = s1; "
                     f"const bool own{u} = true;")
        else:
            b.extend([f"{ind}{IX} l0_{u} = lr0, l1_{u} = lr1, a0_{u} = s0, a1_{u} = s1; "
                  f"bool own{u} = true;",
                  f"{ind}if (r{u} >= nxt0) {{ own{u} = false; int q_ = rg;",
                  f"{ind}  while (q_ + 1 < (int)a.NRG && RG[4 * (q_ + 1)] <= r{u}) ++q_;",
                  f"{ind}  l0_{u} = ({IX})RG[4 * q_]; l1_{u} = ({IX})RG[4 * q_ + 1]; "
                  f"a0_{u} = ({IX})RG[4 * q_ + 2]; a1_{u} = ({IX})RG[4 * q_ + 3]; }}"])
        b.extend([f"{ind}const bool act{u} = in{u} && r{u} < a.NRUNS && r{u} >= l0_{u} && "
              f"r{u} < l1_{u} && a1_{u} > a0_{u};",
              f"{ind}{IX} j{u} = (own{u} && gbase >= 0) ? gbase + {u * 64} + lane : "
              f"a0_{u} + (r{u} - l0_{u});",
              f"{ind}j{u} = act{u} ? (j{u} < a0_{u} ? a0_{u} : (j{u} >= a1_{u} ? a1_{u} - 1 : j{u}))"
              f" : 0;"])
        if lo16 and fast:
            # 16-bit key halves per lane; the full images of the group's two end pairs (lanes
            # 0 / 1 load them for lane 0 / lane 63) decide in ``resolve`` whether halves suffice
            b.extend([f"{ind}const unsigned key{u} = (unsigned)a.LL[act{u} ? r{u} : 0];",
                      f"{ind}const unsigned k{u} = (unsigned)a.RL[j{u}];",
                      f"{ind}const int j0_{u} = __builtin_amdgcn_readlane((int)j{u}, 0), "
                      f"j63_{u} = __builtin_amdgcn_readlane((int)j{u}, 63);",
                      f"{ind}const int re_{u} = (int)((gi + {u}) << 6) + ((lane & 1) ? 63 : 0);",
                      f"{ind}const unsigned fk{u} = (unsigned)a.RK{lk}[re_{u} < a.NRUNS ? re_{u} : 0]"
                      f" + (unsigned)a.KOF;",
                      f"{ind}const unsigned fi{u} = IMGF((lane & 1) ? j63_{u} : j0_{u});"])
        else:
            b.extend([f"{ind}const unsigned key{u} = (unsigned)a.RK{lk}[act{u} ? r{u} : 0] + "
                      f"(unsigned)a.KOF;",
                      f"{ind}const unsigned k{u} = IMGF(j{u});"])
        gu = J._Gen(args, cols, SPLIT, (f"j{u}", f"j{u}"), frozenset(), True)
        for sl in stage_slots:
            J._uload(gu, sl, f"g{u}", b, ind)

    def resolve(u: int, ind: str, lo: bool = False) -> None:
        gu = J._Gen(args, cols, SPLIT, (f"j{u}", f"j{u}"), frozenset(), True)
        # (a checked group's keys are low halves: a miss gallops with the full left key)
        kfull = f"(unsigned)a.RK{lk}[r{u}] + (unsigned)a.KOF" if lo else f"key{u}"
        if lo:
            # halves decide when every lane is active, the guesses are consecutive and both end
            # pairs match in full with a key span below 2^16: any lane's two keys then differ by
            # less than 2^16.  Otherwise every lane takes the full-key path below.
            b.extend([f"{ind}const unsigned fk0_{u} = (unsigned)__builtin_amdgcn_readlane((int)fk{u}, 0), "
                      f"fk1_{u} = (unsigned)__builtin_amdgcn_readlane((int)fk{u}, 1);",
                      f"{ind}const bool cl{u} = __ballot(act{u}) == ~0ull && j63_{u} - j0_{u} == 63 && "
                      f"fk0_{u} == (unsigned)__builtin_amdgcn_readlane((int)fi{u}, 0) && "
                      f"fk1_{u} == (unsigned)__builtin_amdgcn_readlane((int)fi{u}, 1) && "
                      f"fk1_{u} - fk0_{u} < 65536u;",
                      f"{ind}bool hit{u} = act{u} && cl{u} && k{u} == key{u};"])
        else:
            b.append(f"{ind}bool hit{u} = act{u} && k{u} == key{u};")
        b.extend([f"{ind}{IX} m{u} = j{u};",
                  f"{ind}unsigned tg{u} = {tag_expr(gu, f'g{u}', f'hit{u}')};",
                  f"{ind}if (act{u} && !hit{u}) {{",
                  # gallop from the guess to the lower bound of key in [a0, a1)
                  f"{ind}  const unsigned key_ = {kfull}; {IX} lo_, hi_;",
                  f"{ind}  const unsigned kj_ = IMG(j{u});",
                  f"{ind}  if (kj_ == key_) {{ lo_ = j{u}; hi_ = j{u}; }}",
                  f"{ind}  else if (kj_ > key_) {{",
                  f"{ind}    hi_ = j{u}; {IX} st_ = 1; lo_ = j{u} - 1;",
                  f"{ind}    while (lo_ > a0_{u} && IMG(lo_) >= key_) {{ hi_ = lo_; st_ <<= 1; "
                  f"lo_ = hi_ - st_; }}",
                  f"{ind}    if (lo_ < a0_{u}) lo_ = a0_{u};",
                  f"{ind}  }} else {{",
                  f"{ind}    lo_ = j{u} + 1; {IX} st_ = 1; hi_ = j{u} + 1;",
                  f"{ind}    while (hi_ < a1_{u} && IMG(hi_) < key_) {{ lo_ = hi_ + 1; st_ <<= 1; "
                  f"hi_ = j{u} + st_; }}",
                  f"{ind}    if (hi_ > a1_{u}) hi_ = a1_{u};",
                  f"{ind}  }}",
                  f"{ind}  while (lo_ < hi_) {{ const {IX} md_ = (lo_ + hi_) >> 1; "
                  f"if (IMG(md_) < key_) lo_ = md_ + 1; else hi_ = md_; }}",
                  f"{ind}  m{u} = lo_;",
                  f"{ind}  hit{u} = lo_ < a1_{u} && IMG(lo_) == key_;",
                  f"{ind}  const {IX} jm{u} = hit{u} ? lo_ : 0;"])
        gm = J._Gen(args, cols, SPLIT, (f"jm{u}", f"jm{u}"), frozenset(), True)
        for sl in stage_slots:
            J._uload(gm, sl, f"h{u}", b, ind + "  ")
        b.extend([f"{ind}  tg{u} = {tag_expr(gm, f'h{u}', f'hit{u}')};",
                  f"{ind}}}"])
        # the group's 2W tag words: whole words, plain stores
        if W == 1:
            b.extend([f"{ind}{{ const u64 bal_ = __ballot(tg{u} != 0u);",
                      f"{ind}  if (in{u} && lane < 2) a.tags[((gi + {u}) << 1) + lane] = "
                      f"(unsigned)(bal_ >> (32 * lane)); }}"])
        else:
            per_w = 32 // W
            b.extend([f"{ind}{{ unsigned wd_ = 0u;",
                      f"{ind}  for (int i_ = 0; i_ < {per_w}; ++i_) {{",
                      f"{ind}    const int src_ = ((lane * {per_w}) + i_) & 63;",
                      f"{ind}    wd_ |= (((unsigned)__shfl((int)tg{u}, src_, 64)) & {MASK}u) << "
                      f"(unsigned)(i_ * {W}); }}",
                      f"{ind}  if (in{u} && lane < {2 * W}) a.tags[(gi + {u}) * {2 * W} + lane] = "
                      f"wd_; }}"])
        if mode == "rec":
            b.append(f"{ind}if (in{u} && r{u} < a.NRUNS) a.MOUT[r{u}] = hit{u} ? (int)m{u} : -1;")

    def iteration(fast: bool, ind: str) -> None:
        for u in range(U):
            group(u, fast, ind)
        for u in range(U):
            resolve(u, ind, lo16 and fast)
        # next iteration's guess: the last group's last lane, when it matched in this range
        b.extend([f"{ind}{{ const {IX} nx_ = __shfl((hit{U - 1} && own{U - 1}) ? m{U - 1} + 1 : "
                  f"({IX})-1, 63, 64);",
                  f"{ind}  gbase = nx_; }}"])
    iteration(True, ind)
    b.append("    } else {   // a range starts inside this iteration's groups")
    iteration(False, ind)
    b += ["    }", "  }"]
    src = (J._PRELUDE + args.struct_src() +
           f'extern "C" __global__ __launch_bounds__({J.BLOCK}) void hs_jit_run_tags2(Args a) {{\n' +
           "\n".join(b) + "\n}\n")
    return J.Kernel(src, "hs_jit_run_tags2", args)


def _tag_stores(b: List[str], u: int, W: int, ind: str) -> None:
    """The 2W tag words of 64-run group ``gi + u`` from the lanes' tags ``tg<u>``: whole words,
    plain stores."""
    if W == 1:
        b.extend([f"{ind}{{ const u64 bal_ = __ballot(tg{u} != 0u);",
                  f"{ind}  if (in{u} && lane < 2) a.tags[((gi + {u}) << 1) + lane] = "
                  f"(unsigned)(bal_ >> (32 * lane)); }}"])
        return
    per_w = 32 // W
    b.extend([f"{ind}{{ unsigned wd_ = 0u;",
              f"{ind}  for (int i_ = 0; i_ < {per_w}; ++i_) {{",
              f"{ind}    const int src_ = ((lane * {per_w}) + i_) & 63;",
              f"{ind}    wd_ |= (((unsigned)__shfl((int)tg{u}, src_, 64)) & {(1 << W) - 1}u) << "
              f"(unsigned)(i_ * {W}); }}",
              f"{ind}  if (in{u} && lane < {2 * W}) a.tags[(gi + {u}) * {2 * W} + lane] = wd_; }}"])


def copy_ok(p: NL.JoinParams, compacts) -> bool:
    """Whether phase 1 can read per-run copies of its right columns (mode "copy"): every staged
    column is stored plainly or as a one-array compact code (not the grouped 16-bit form)."""
    cols = J._col_specs(p, compacts)
    for sl in _stage_slots(p):
        enc = cols[sl][2]
        if enc and len(enc) > 2 and enc[2] == 64:
            return False
    return True


def _gen_tags2_match(p: NL.JoinParams, compacts, W: int, copy: bool = False) -> J.Kernel:
    """Phase 1 over a recorded match (``gen_run_tags2`` mode "match"): per run one int32 load
    of its right row (-1: no match, or the run is outside the lowering's ranges), then the right
    predicate / group columns at that row.  No key images, no range table, no gallop: the
    record already resolved them (``record_matches``), so the phase reads 4 bytes per run plus
    the staged right columns (monotone rows: coalesced).

    ``copy`` (mode "copy"): the right columns were gathered into run order at the record
    (``S<slot>`` / ``SV<slot>``, ``gen_match_gather``) and the match is one bit per run
    (``HIT``, one 64-bit word per 64-run group, read once per wavefront): the phase reads the
    stored codes of its predicate columns per run and nothing at right rows."""
    args = J.Args()
    if copy:
        args.add("p", "HIT", "const u64*")
    else:
        args.add("p", "MATCH", "const int*")
    args.add("p", "tags", "unsigned*")
    args.add("q", "NRUNS", "long long")
    cols = J._col_specs(p, compacts)
    rpreds = _rpreds(p)
    rgroup = _tags_grouped(p)
    stage_slots = _stage_slots(p)
    if rgroup:
        gb = args.add("q", "group_base", "long long")
        ng = args.add("q", "num_groups", "long long")
    U = max(1, RT2_UNROLL)  # noqa: N806
    WV = J.BLOCK // 64  # noqa: N806
    ind = "    "
    b: List[str] = [
        "  const int lane = (int)(threadIdx.x & 63);",
        "  const i64 G = (a.NRUNS + 63) >> 6;",
        f"  const i64 nwv = (i64)gridDim.x * {WV};",
        f"  const i64 wv = (i64)blockIdx.x * {WV} + "
        "(i64)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));",
        "  const i64 per = (G + nwv - 1) / nwv;",
        "  const i64 gbeg = wv * per;",
        "  const i64 gend = G < gbeg + per ? G : gbeg + per;",
        f"  for (i64 gi = gbeg; gi < gend; gi += {U}) {{"]
    for u in range(U):
        # the record is padded to whole groups: an in-range group's 64 lanes all read it
        b.append(f"{ind}const bool in{u} = gi + {u} < gend;")
        if copy:
            b.extend([f"{ind}const int r{u} = in{u} ? (int)(((gi + {u}) << 6) + lane) : lane;",
                      f"{ind}const u64 hb{u} = a.HIT[in{u} ? gi + {u} : 0];"])
            for sl in stage_slots:
                gt = J._Gen(args, cols, SPLIT, ("r_", "r_"), frozenset(), True)
                sp = args.add("p", f"S{sl}", f"const {gt.raw_type(sl)}*")
                b.append(f"{ind}const {gt.raw_type(sl)} w{sl}_g{u} = {sp}[r{u}];")
                if cols[sl][1]:
                    vp = args.add("p", f"SV{sl}", "const unsigned char*")
                    b.append(f"{ind}const unsigned char u{sl}_g{u} = {vp}[r{u}];")
        else:
            b.append(f"{ind}const int mt{u} = a.MATCH[in{u} ? (((gi + {u}) << 6) + lane) : lane];")
    for u in range(U):
        if copy:
            b.append(f"{ind}const bool hit{u} = in{u} && ((hb{u} >> lane) & 1ull);")
            gu = J._Gen(args, cols, SPLIT, (f"r{u}", f"r{u}"), frozenset(), True)
            for sl in stage_slots:
                J._uload_raw(gu, sl, f"g{u}", f"w{sl}_g{u}", f"u{sl}_g{u}", b, ind)
            continue
        b.extend([f"{ind}const bool hit{u} = in{u} && mt{u} >= 0;",
                  f"{ind}const int j{u} = hit{u} ? mt{u} : 0;"])
        gu = J._Gen(args, cols, SPLIT, (f"j{u}", f"j{u}"), frozenset(), True)
        for sl in stage_slots:
            J._uload(gu, sl, f"g{u}", b, ind)
    for u in range(U):
        gu = J._Gen(args, cols, SPLIT, (f"j{u}", f"j{u}"), frozenset(), True)
        cond = J._rename(gu.cnf(rpreds), stage_slots, f"g{u}")
        if rgroup:
            gx = J._rename(f"x{p.group_col}", stage_slots, f"g{u}")
            b.append(f"{ind}const unsigned tg{u} = ({{ const i64 gl_ = (i64){gx} - {gb}; "
                     f"(hit{u} && {cond} && gl_ >= 0 && gl_ < {ng}) ? (unsigned)(gl_ + 1) : 0u; }});")
        else:
            b.append(f"{ind}const unsigned tg{u} = (hit{u} && {cond}) ? 1u : 0u;")
        _tag_stores(b, u, W, ind)
    b.append("  }")
    src = (J._PRELUDE + args.struct_src() +
           f'extern "C" __global__ __launch_bounds__({J.BLOCK}) void hs_jit_run_tags2(Args a) {{\n' +
           "\n".join(b) + "\n}\n")
    return J.Kernel(src, "hs_jit_run_tags2", args)


def record_matches(p: NL.JoinParams, compacts, W: int, vt: dict, nruns: int, grid: int, dev):
    """Each run's matched right row under the lowering's ranges (or -1), padded with -1 to whole
    64-run groups: one launch of the verifying phase 1 in mode "rec" at lowering time (queued on
    the current stream).  Literal-independent: the ranges, key frame and key columns are fixed
    for the launcher, and the record mode stores the match before any right predicate."""
    import torch
    m = torch.full((((nruns + 63) >> 6) * 64,), -1, dtype=torch.int32, device=dev)
    kr = J.kernel_for(tags2_shape(p, compacts, W, True, "rec"),
                      lambda: gen_run_tags2(p, compacts, W, True, "rec"))
    v = dict(vt)
    v["MOUT"] = m.data_ptr()
    J.fill_preds_aggs(v, [(k_, p.preds[k_]) for k_ in range(p.npreds)], [], compacts)
    kr.launch(grid, v, NL.stream_ptr(), 0)
    return m


def gen_match_gather(p: NL.JoinParams, compacts) -> J.Kernel:
    """The right columns phase 1 reads, gathered into run order at the recorded match
    (``S<slot>`` stored elements, ``SV<slot>`` validity bytes; row 0 for a run without one - its
    HIT bit is clear): one pass at record time for the "copy" form of phase 1."""
    args = J.Args()
    args.add("p", "MATCH", "const int*")
    args.add("q", "N", "long long")
    cols = J._col_specs(p, compacts)
    g = J._Gen(args, cols, SPLIT, ("j_", "j_"), frozenset(), True)
    b = [f"  for (i64 i = (i64)blockIdx.x * {J.BLOCK} + threadIdx.x; i < a.N; "
         f"i += (i64)gridDim.x * {J.BLOCK}) {{",
         "    const int m_ = a.MATCH[i]; const int j_ = m_ >= 0 ? m_ : 0;"]
    for sl in _stage_slots(p):
        sp = args.add("p", f"S{sl}", f"{g.raw_type(sl)}*")
        b.append(f"    {sp}[i] = {g.ptr(sl)}[j_];")
        if cols[sl][1]:
            vp = args.add("p", f"SV{sl}", "unsigned char*")
            b.append(f"    {vp}[i] = {g.vptr(sl)}[j_];")
    b.append("  }")
    src = (J._PRELUDE + args.struct_src() +
           f'extern "C" __global__ __launch_bounds__({J.BLOCK}) void hs_jit_match_gather(Args a) '
           "{\n" + "\n".join(b) + "\n}\n")
    return J.Kernel(src, "hs_jit_match_gather", args)


def copy_matches(p: NL.JoinParams, compacts, m, vt: dict, dev) -> tuple:
    """From a recorded match ``m``: the HIT words (bit l of word g: run 64 g + l has a right
    row) and the gathered right columns; returns (tensors to keep, their argument values)."""
    import torch
    n = int(m.numel())
    hit = ((m.view(-1, 64) >= 0).to(torch.int64) <<
           torch.arange(64, device=dev, dtype=torch.int64)).sum(1)  # distinct bits: sum == OR
    keep, vals = [hit], {"HIT": hit.data_ptr()}
    cols = J._col_specs(p, compacts)
    g = J._Gen(J.Args(), cols, SPLIT, ("j_", "j_"), frozenset(), True)
    for sl in _stage_slots(p):
        t = torch.empty(n * J._SIZEOF[g.raw_type(sl)], dtype=torch.uint8, device=dev)
        keep.append(t)
        vals[f"S{sl}"] = t.data_ptr()
        if cols[sl][1]:
            v = torch.empty(n, dtype=torch.uint8, device=dev)
            keep.append(v)
            vals[f"SV{sl}"] = v.data_ptr()
    kg = J.kernel_for(("match_gather", tags2_shape(p, compacts, 1)[1], tuple(_stage_slots(p)),
                       J.BLOCK),
                      lambda: gen_match_gather(p, compacts))
    a = dict(vt, MATCH=m.data_ptr(), N=n, **vals)
    kg.launch(max(1, min(8192, (n + J.BLOCK - 1) // J.BLOCK)), a, NL.stream_ptr(), 0)
    return keep, vals


def lo16_keys(p: NL.JoinParams, compacts, W: int, vt: dict, nruns: int, nright: int, grid: int,
              dev):
    """The low 16 bits of the left run key images and the right key images (phase 1's checked
    groups compare these: ``gen_run_tags2`` mode "lo16"), computed once per reused lowering;
    None when the right key has nulls (a null's image 0 could alias a left key's low half).
    Literal-independent encodings of the key columns: every query still matches its keys."""
    import torch
    from .device_cache import track_derived
    if J._col_specs(p, compacts)[p.rkey][1]:
        return None
    ll = torch.empty(max(nruns, 1), dtype=torch.int16, device=dev)
    rl = torch.empty(max(nright, 1), dtype=torch.int16, device=dev)
    kp = J.kernel_for(tags2_shape(p, compacts, W, True, "lo16prep"),
                      lambda: gen_run_tags2(p, compacts, W, True, "lo16prep"))
    kp.launch(grid, dict(vt, LL=ll.data_ptr(), RL=rl.data_ptr(), NRIGHT=nright),
              NL.stream_ptr(), 0)
    track_derived(ll)
    track_derived(rl)
    return ll, rl


def run_ranges(rstart, rlen, rbucket, roff, runs):
    """RNG of ``gen_run_tags2``: per non-empty left row range (first run, end run, right bucket
    rows [s0, s1)), sorted by first run; computed once per lowering (one small D2H)."""
    import numpy as np
    import torch
    rs = rstart.cpu().numpy().astype(np.int64)
    rl = rlen.cpu().numpy().astype(np.int64)
    rb = rbucket.cpu().numpy().astype(np.int64)
    ro = roff.cpu().numpy().astype(np.int64)
    keep = rl > 0
    rs, rl, rb = rs[keep], rl[keep], rb[keep]
    if len(rs) == 0:
        return np.zeros((0, 4), np.int64)
    rows = np.concatenate([rs, rs + rl - 1])
    gi = torch.from_numpy(rows >> 6).to(runs.gmask.device)
    gm = runs.gmask.index_select(0, gi).cpu().numpy().view(np.uint64)
    gr = runs.gruns.index_select(0, gi).cpu().numpy().astype(np.int64)
    full = (1 << 64) - 1
    # run of a row: the group's first run + run starts among the group's rows 1..i
    run = np.array([int(g_) + bin(int(m_) & (((2 << int(r_ & 63)) - 2) & full)).count("1")
                    for g_, m_, r_ in zip(gr, gm, rows)], dtype=np.int64)
    n = len(rs)
    out = np.stack([run[:n], run[n:] + 1, ro[rb], ro[rb + 1]], axis=1)
    return out[np.argsort(out[:, 0], kind="stable")]


def scan_shape(p: NL.JoinParams, compacts, W: int, NI: int) -> tuple:
    cols = tuple(sorted((s, c) for s, c in J._col_specs(p, compacts).items() if s < SPLIT))
    preds = tuple((p.preds[k].kind, p.preds[k].op, p.preds[k].col, p.preds[k].col2,
                   p.preds[k].group) for k in range(p.nlp))
    aggs = tuple((p.aggs[i].kind, p.aggs[i].nterms, tuple(p.aggs[i].col[:p.aggs[i].nterms]))
                 for i in range(p.naggs))
    return ("run_scan", cols, preds, aggs, p.group_col, p.lkey, W, NI, J.BLOCK, J.WAVE_SYNC,
            J.VEC_PREFETCH, _scan_grouped(p))


def _scan_grouped(p: NL.JoinParams) -> bool:
    """Whether the scan phase keeps a group table: a right-side group key with a single group
    (a constant column) accumulates like an ungrouped aggregate (same partials layout)."""
    return p.group_col >= 0 and not (p.group_col >= SPLIT and p.num_groups == 1)


def gen_run_scan(p: NL.JoinParams, compacts, W: int, NI: int) -> J.Kernel:
    """Phase 2 (module docstring): the left rows' scan with the run-tag test."""
    args = J.Args()
    for n, ct in (("rstart", "const long long*"), ("rlen", "const long long*"),
                  ("tile_prefix", "const long long*")):
        args.add("p", n, ct)
    lk = p.lkey
    args.add("p", f"GM{lk}", "const unsigned long long*")
    args.add("p", f"GR{lk}", "const int*")
    args.add("p", "tags", "const unsigned*")
    args.add("q", "R", "long long")
    args.add("q", "nrows", "long long")
    J._common_args(args)
    cols = J._col_specs(p, compacts)
    lpreds = _lpreds(p)
    aggs = [p.aggs[i] for i in range(p.naggs)]
    grouped = _scan_grouped(p)
    rgroup = grouped and p.group_col >= SPLIT
    pslots = J._pred_slots(lpreds)
    tail = J._agg_slots(aggs) + ([p.group_col] if grouped and not rgroup else [])
    allslots = list(dict.fromkeys(pslots + tail))
    approx = J._sum_only_slots(lpreds, aggs, p.group_col if grouped and not rgroup else -1, cols)
    BLOCK = J.BLOCK  # noqa: N806
    T = BLOCK * NI  # noqa: N806
    MASK = (1 << W) - 1  # noqa: N806
    KW = ((31 + (NI - 1) * W) >> 5) + 1  # noqa: N806 — tag words a thread's rows can touch
    ind = "    "
    g1 = J._Gen(args, cols, SPLIT, ("row0", "row0"), approx, True)
    b: List[str] = []
    b += J._acc_decls(aggs, grouped, args)

    def body(b: List[str], full: bool) -> None:
        J._vec_load_slots(b, g1, pslots, NI, ind)
        for it in range(NI):
            gi = J._Gen(args, cols, SPLIT, (f"row{it}", f"row{it}"), approx, True)
            b.append(f"{ind}bool pass{it} = act{it} && "
                     f"{J._rename(gi.cnf(lpreds), allslots, it)};")
        # row -> run: the thread's NI rows lie in one 64-row group (NI | 64, g0 % NI == 0)
        b += [f"{ind}const int sh_ = (int)(g0 & 63);",
              f"{ind}const i64 r0_ = (i64)gr_ + (i64)__popcll(gm_ & ((2ull << sh_) - 2ull));",
              f"{ind}const unsigned gl_ = (unsigned)(gm_ >> sh_);",
              f"{ind}const i64 b0_ = r0_ * {W};",
              f"{ind}const i64 w0_ = b0_ >> 5;",
              f"{ind}" + " ".join(f"const unsigned tw{k}_ = a.tags[w0_ + {k}];" for k in range(KW))]
        for it in range(NI):
            ri = "0" if it == 0 else f"(int)__popc(gl_ & {(2 << it) - 2}u)"
            b.append(f"{ind}{{ const int rel = (int)(b0_ & 31) + {ri} * {W};")
            sel = f"tw{KW - 1}_"
            for k in reversed(range(KW - 1)):
                sel = f"((rel >> 5) == {k} ? tw{k}_ : {sel})"
            b += [f"{ind}  const unsigned tg = ({sel} >> (unsigned)(rel & 31)) & {MASK}u;",
                  f"{ind}  pass{it} = pass{it} && tg != 0u;",
                  f"{ind}  jg{it} = (int)tg - 1; }}"]
        b.extend(J._compacted_tail(args, cols, SPLIT, approx, aggs, grouped, p.group_col,
                                   tail, allslots, NI, ind, with_j=rgroup, j_fmt="jg{it}",
                                   jgroup=rgroup))

    def body_decl(b: List[str], full: bool) -> None:
        b.append(f"{ind}int " + ", ".join(f"jg{it} = 0" for it in range(NI)) + ";")
        body(b, full)

    gi = "((G0 < a.nrows ? G0 : a.nrows - 1) >> 6)"
    J._vec_tiles(b, T, NI, ind, J._vec_loads(g1, pslots),
                 [("gm_", "unsigned long long", f"a.GM{lk}[{gi}]"),
                  ("gr_", "int", f"a.GR{lk}[{gi}]")], body_decl)
    b += ["  }"]
    b += J._flush(aggs, grouped)
    Wv = BLOCK // 64  # noqa: N806
    pre = [f"  typedef {J._crow_t(T)} crow_t; __shared__ crow_t crow_s[{Wv}][{64 * NI}];",
           "  const int cln = threadIdx.x & 63, wv = threadIdx.x >> 6;"]
    if rgroup:
        pre.append(f"  __shared__ int cj_s[{Wv}][{64 * NI}];")
    src = (J._PRELUDE + args.struct_src() +
           f'extern "C" __global__ __launch_bounds__({BLOCK}) void hs_jit_run_scan(Args a) {{\n' +
           "\n".join(pre + b) + "\n}\n")
    lds = (len(aggs) * p.num_groups * 32) if grouped else 0
    return J.Kernel(src, "hs_jit_run_scan", args, lds)


# phase 2 for 1-bit tags: masks 64 rows at a time (gen_run_sparse_scan; RS_BITS), aggregate
# inputs read row-packed when they fit one 64-bit word (pack_layout / packed_tail; RS_PACK).  (A
# row-mask expansion between the phases with a gated dense scan measured no faster: removed.)


def _tail_slots(p: NL.JoinParams) -> list:
    grouped = _scan_grouped(p)
    aggs = [p.aggs[i] for i in range(p.naggs)]
    return list(dict.fromkeys(J._agg_slots(aggs) + ([p.group_col] if grouped else [])))


def pack_layout(p: NL.JoinParams, compacts) -> Optional[tuple]:
    """((slot, bit offset, code bytes), ...) of the row-packed aggregate inputs of the bits
    scan: two or more compact-coded tail columns without validity whose codes fit 64 bits."""
    if not RS_PACK:
        return None
    slots = _tail_slots(p)
    if len(slots) < 2:
        return None
    out, off = [], 0
    for sl in slots:
        c = (compacts or {}).get(sl)
        if c is None or p.cols[sl].valid or getattr(c, "runs", None) or \
                type(c).__name__ != "Compact" or c.width not in (1, 2, 4):
            return None
        out.append((sl, off, c.width))
        off += 8 * c.width
    return tuple(out) if off <= 64 else None


# (ids of the packed code tensors) -> (the tensors, packed int64 words): derived per resident
# table once, like the compact codes themselves
_PACKS: dict = {}


def packed_tail(layout, compacts):
    """One int64 word per row: each layout column's code at its bit offset (uint bits)."""
    import torch
    key = tuple(id(compacts[sl].codes) for sl, _, _ in layout)
    hit = _PACKS.get(key)
    if hit is not None and all(a is compacts[sl].codes for a, (sl, _, _) in zip(hit[0], layout)):
        return hit[1]
    n = compacts[layout[0][0]].codes.numel()
    w = torch.zeros(n, dtype=torch.int64, device=compacts[layout[0][0]].codes.device)
    for sl, off, nb in layout:
        c = compacts[sl].codes.to(torch.int64) & ((1 << (8 * nb)) - 1)
        w |= c << off
        del c
    if len(_PACKS) >= 8:
        _PACKS.pop(next(iter(_PACKS)))
    _PACKS[key] = (tuple(compacts[sl].codes for sl, _, _ in layout), w)
    return w


# 12-bit packed copies of 16-bit predicate codes (the bits scan's row stream): 64 rows in 24
# dwords, 8 rows per 3 dwords (value j at bits [12 j, 12 j + 12) of the 96-bit chunk) - 25% fewer
# bytes for the one column phase 2 reads for every row.  Derived once per resident table (like
# the compact codes and the row-packed aggregate inputs), kept while its codes are.
_P12: dict = {}


def _p12_offset(c) -> int:
    """The smallest code of compact column ``c`` (codes = value - base, values in [lo, hi])."""
    return int(c.lo) - int(c.base)


def pack12_ok(c) -> bool:
    """Whether compact column ``c``'s codes are 16-bit and span at most 4096 values (host
    metadata): the packed copy stores code - (lo - base) in 12 bits."""
    if c is None or type(c).__name__ != "Compact" or c.width != 2 or getattr(c, "runs", None):
        return False
    if c.lo is None or c.hi is None:
        return False
    return 0 <= int(c.hi) - int(c.lo) <= 4095


def packed12(c):
    """The 12-bit packed copy of compact column ``c`` (``pack12_ok``), cached per codes tensor."""
    import torch
    key = id(c.codes)
    hit = _P12.get(key)
    if hit is not None and hit[0] is c.codes:
        return hit[1]
    n = c.codes.numel()
    npad = (n + 63) // 64 * 64
    v = torch.zeros(npad, dtype=torch.int64, device=c.codes.device)
    v[:n] = (c.codes.to(torch.int64) - _p12_offset(c)) & 0xFFF
    v = v.view(-1, 8)
    a = v[:, 0] | (v[:, 1] << 12) | ((v[:, 2] & 0xFF) << 24)
    b = (v[:, 2] >> 8) | (v[:, 3] << 4) | (v[:, 4] << 16) | ((v[:, 5] & 0xF) << 28)
    cc = (v[:, 5] >> 4) | (v[:, 6] << 8) | (v[:, 7] << 20)
    w = torch.stack([a, b, cc], dim=1).reshape(-1)
    w = torch.where(w >= (1 << 31), w - (1 << 32), w).to(torch.int32).contiguous()
    del v, a, b, cc
    if len(_P12) >= 8:
        _P12.pop(next(iter(_P12)))
    _P12[key] = (c.codes, w)
    return w


def _p12_slots(p: NL.JoinParams, compacts) -> tuple:
    """Predicate slots of phase 2 that read a 12-bit packed copy (RS_PACK12), or ()."""
    if not RS_PACK12 or not RS_PK16:
        return ()
    slots = J._pred_slots(_lpreds(p))
    if not slots or any(p.cols[sl].valid or not pack12_ok((compacts or {}).get(sl))
                        for sl in slots):
        return ()
    # every leaf must have the packed range-test form (Gen.cnf_sign2)
    for _, pr in _lpreds(p):
        if pr.kind == NL.PK_TRUE:
            continue
        c = (compacts or {}).get(pr.col)
        scaled = c is not None and c.scale is not None
        if pr.col not in slots or pr.kind not in (NL.PK_INT_LIT, NL.PK_FLT_LIT, NL.PK_IS_NULL,
                                                   NL.PK_NOT_NULL):
            return ()
        if (pr.kind == NL.PK_INT_LIT and scaled) or (pr.kind == NL.PK_FLT_LIT and not scaled):
            return ()
    return tuple(slots)


def fill_pack12(vs: dict, p: NL.JoinParams, compacts) -> list:
    """The packed copies' pointers into a phase-2 argument dict; returns the tensors to keep."""
    keep = []
    for sl in _p12_slots(p, compacts):
        w = packed12(compacts[sl])
        vs[f"P12_{sl}"] = w.data_ptr()
        vs[f"P12O_{sl}"] = _p12_offset(compacts[sl])
        keep.append(w)
    return keep


def sparse_shape(p: NL.JoinParams, compacts, hk=None, tk=None) -> tuple:
    return ("run_bits_scan", RS_PIPE, RS_WALK, RS_LDS, RS_LUT, RS_PK16, RS_WAVES,
            _p12_slots(p, compacts)) + scan_shape(p, compacts, 1, 64)[1:] + \
        (pack_layout(p, compacts),) + ((hk.shape(),) if hk is not None else ()) + \
        ((tk.shape(),) if tk is not None else ())


def gen_run_sparse_scan(p: NL.JoinParams, compacts, hk=None, tk=None) -> J.Kernel:
    """Phase 2 for 1-bit tags, bit-parallel: the dense per-row scan spends ~20 VALU
    instructions per row (decode, predicate, run index by popcount, tag extract, compaction
    ballot + mbcnt), which bounds it below HBM speed.  Here a wavefront takes 4096-row tiles of
    the left ranges, lane l the 64-row group l of its tile, and works on 64-bit row masks:

    1. tag mask: the tag bits of the group's runs (gruns / 3 tag words) deposited at the run
       starts (gmask) and spread over each run's rows by a prefix XOR (as hs_run_rowmask),
       limited to the tile's range rows - ~1.5 instructions per row;
    2. predicate mask: the lane's 64 rows of every left predicate column (vector loads, in
       flight with the tag words), one compare + shift-or per row;
    3. the rows of (tag mask & predicate mask) - the join's passing rows, a few percent - go to
       a per-wavefront LDS list (offsets from a shuffle scan of the lanes' popcounts), which the
       wavefront walks 4 entries per lane per pass: aggregate inputs loaded at those rows only
       and accumulated.

    The next tile's run-form words are prefetched during the current tile.

    With ``hk`` (an exec.hash_agg.KeyPlan over left columns) the walk groups by the hash key
    instead: each pass's 64 list entries are consecutive passing rows, so a segmented shuffle
    reduce folds a group's rows (one run = one left join key) before one table probe
    (``jit_hash._hash_accumulate``); kernel ``hs_jit_run_bits_hash``, no partials.

    With ``tk`` as well (an exec.hash_agg.TopKPlan: ORDER BY <aggregate> LIMIT k over those
    groups), the windows are walked in row order with the last segment of each carried into
    the next (``jit_hash._topk_accumulate``): a key is final when the walk leaves it and competes
    for the wavefront's top-K registers instead of probing the table; only keys that may
    continue into the neighbouring wavefronts' tiles (at most two per wavefront) go to the
    table (kernel ``hs_jit_run_bits_topk``; every wavefront writes its list at the end)."""
    args = J.Args()
    for n, ct in (("rstart", "const long long*"), ("rlen", "const long long*"),
                  ("tile_prefix", "const long long*")):
        args.add("p", n, ct)
    lk = p.lkey
    args.add("p", f"GM{lk}", "const unsigned long long*")
    args.add("p", f"GR{lk}", "const int*")
    args.add("p", "tags", "const unsigned*")
    args.add("q", "R", "long long")
    args.add("q", "nrows", "long long")
    J._common_args(args)
    cols = J._col_specs(p, compacts)
    lpreds = _lpreds(p)
    aggs = [p.aggs[i] for i in range(p.naggs)]
    grouped = _scan_grouped(p)
    assert not (grouped and p.group_col >= SPLIT)
    pslots = J._pred_slots(lpreds)
    assert not (grouped and hk is not None)
    # top-K mode segments the walk by key run (lrn_) and loads the key columns only where a
    # group is emitted (jit_hash._hash_accumulate ``seg``): they are not part of the per-row tail
    tail = list(dict.fromkeys(J._agg_slots(aggs) + ([p.group_col] if grouped else []) +
                              (list(hk.slots) if hk is not None and tk is None else [])))
    approx = J._sum_only_slots(lpreds, aggs, p.group_col if grouped else -1, cols) - \
        set(hk.slots if hk is not None else [])
    BLOCK = J.BLOCK  # noqa: N806
    WV = BLOCK // 64  # noqa: N806
    T = 4096  # noqa: N806 — rows per wavefront tile: 64 groups, one per lane
    NI = 64  # noqa: N806
    b: List[str] = []
    b += J._acc_decls(aggs, grouped, args)
    assert tk is None or hk is not None
    if tk is not None:
        b += JH._topk_decls(aggs, tk)
    CAP = 1024  # noqa: N806 — list entries per wavefront and round (a denser tile takes rounds)
    EW = max(1, RS_WALK)  # noqa: N806 — list entries per lane per walk pass, loads in flight together

    def geom(tv: str, sfx: str) -> List[str]:
        """Tile ``tv``'s range / row geometry and its group's run-form words (suffix sfx).  The
        words stay in their loaded types (no OR / widening here): an operation on a loaded value
        makes the compiler wait for the load on the spot, and these are prefetched a tile ahead."""
        return [f"    while (r + 1 < (int)a.R && a.tile_prefix[r + 1] <= {tv}) ++r;",
                f"    rs{sfx} = a.rstart[r]; re{sfx} = rs{sfx} + a.rlen[r];",
                f"    tb{sfx} = (rs{sfx} & ~(i64)63) + ({tv} - a.tile_prefix[r]) * {T};",
                f"    {{ const i64 r0_ = tb{sfx} + 64 * ln; "
                f"const i64 g_ = (r0_ < a.nrows ? r0_ : a.nrows - 1) >> 6;",
                f"      gm{sfx} = a.GM{lk}[g_]; gr{sfx} = a.GR{lk}[g_]; }}"]
    if tk is not None:
        b.append(f"  __shared__ unsigned short lrn_[{WV}][{CAP}];")
    if RS_LUT:
        # dlut_[m | w << 4]: the 4 row tags of a nibble with run-start bits m, tag window w
        b += ["  __shared__ unsigned char dlut_[512];",
              f"  for (int e_ = (int)threadIdx.x; e_ < 512; e_ += {BLOCK}) {{",
              "    unsigned k_ = 0u, o_ = 0u;",
              "    for (int j_ = 0; j_ < 4; ++j_) { k_ += (e_ >> j_) & 1; "
              "o_ |= (((unsigned)e_ >> (4u + k_)) & 1u) << j_; }",
              "    dlut_[e_] = (unsigned char)o_; }",
              "  __syncthreads();"]
    b += [f"  __shared__ unsigned short lst_[{WV}][{CAP}];",
          "  const int ln = (int)(threadIdx.x & 63);",
          "  const int wq = (int)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));",
          "  const i64 ntiles = a.tile_prefix[a.R];",
          f"  const i64 nwv = (i64)gridDim.x * {WV};",
          f"  const i64 wid = (i64)blockIdx.x * {WV} + wq;",
          "  const i64 per = (ntiles + nwv - 1) / nwv;",
          "  const i64 t0 = wid * per;",
          "  const i64 t1 = ntiles < t0 + per ? ntiles : t0 + per;",
          "  int r = 0;",
          "  if (t0 < t1) { int lo = 0, hi = (int)a.R;",
          "    while (hi - lo > 1) { const int m = (lo + hi) >> 1; "
          "if (a.tile_prefix[m] <= t0) lo = m; else hi = m; }",
          "    r = lo; }",
          # software pipeline (RS_PIPE), one exposed memory round trip per tile: tile t's tag
          # words and predicate columns were issued during tile t-1 (after its masks were
          # formed, before its list walk, so the walk's aggregate-input loads wait on them
          # together) and the run-form words of tile t+1 one tile earlier still (the tag words'
          # address needs them).  The tile loop is unrolled by two over two named buffers (A, B):
          # a loop-carried array is copied register to register at the back edge otherwise,
          # after a wait for its loads, and held twice.
          "  i64 rsC = 0, reC = 0, tbC = 0; u64 gmC = 0ull; int grC = 0;",
          "  i64 rsN = 0, reN = 0, tbN = 0; u64 gmN = 0ull; int grN = 0;",
          "  unsigned tw0A_ = 0u, tw1A_ = 0u, tw2A_ = 0u, tw0B_ = 0u, tw1B_ = 0u, tw2B_ = 0u;"]
    g1 = J._Gen(args, cols, SPLIT, ("row0", "row0"), approx, True)
    elem = {}   # array name -> C expression of element (idx) from its packed 32-bit words
    issue = []  # the current tile's (C) tag-word and predicate-column loads into buffer @S@
    xpose = []  # RS_LDS: the loaded columns' chunks moved to their rows' lanes
    slab = 0    # RS_LDS: 16-byte LDS slots per wavefront
    issue.append("    { const i64 w_ = (i64)grC >> 5; tw0@S@_ = a.tags[w_]; "
                 "tw1@S@_ = a.tags[w_ + 1]; tw2@S@_ = a.tags[w_ + 2]; }")
    p12 = _p12_slots(p, compacts)
    for sl in p12:
        # 24 dwords (96 bytes) per lane: its 64-row group's 12-bit packed codes
        pp = args.add("p", f"P12_{sl}", "const unsigned*")
        args.add("q", f"P12O_{sl}", "long long")
        b.append(f"  unsigned x{sl}qA[24], x{sl}qB[24];")
        issue.append(f"    bload<24>(hs_rsrc((const char*){pp} + (tbC >> 6) * 96, "
                     f"@LIVE@((a.nrows + 63 - tbC) >> 6) * 96), (unsigned)(ln * 96), x{sl}q@S@);")
    for name, ct, ptr in ([] if p12 else J._vec_loads(g1, pslots)):
        es = J._SIZEOF[ct]
        nw = NI * es // 4
        per = 4 // es
        b.append(f"  unsigned {name}wA[{nw}], {name}wB[{nw}];")
        # the group's rows past the table end read as 0 (buffer range check); they are outside
        # every row range, so the range mask drops them
        if RS_LDS:
            issue.append(f"    bload_t<{nw}>(hs_rsrc((const char*){ptr} + tbC * {es}, "
                         f"@LIVE@(a.nrows - tbC) * {es}), ln, {name}w@S@);")
            xpose.append(f"    hs_lds_t<{nw}>(&xt_[wq][0], ln, {name}w@S@);")
            slab = max(slab, nw // 4 * 64)
        else:
            issue.append(f"    bload<{nw}>(hs_rsrc((const char*){ptr} + tbC * {es}, "
                         f"@LIVE@(a.nrows - tbC) * {es}), (unsigned)(64 * ln * {es}), "
                         f"{name}w@S@);")
        elem[name] = (ct, f"{name}w@S@[({{i}}) / {per}]" if per > 1 else f"{name}w@S@[{{i}}]",
                      8 * es, per)

    def buf(lines: List[str], sfx: str) -> List[str]:
        return [x.replace("@S@", sfx).replace("@LIVE@", "") for x in lines]

    b.append("  if (t0 < t1) {")
    if RS_PIPE:
        b += geom("t0", "C")
        b += buf(issue, "A")
        b += ["    if (t0 + 1 < t1) {"]
        b += ["  " + x for x in geom("(t0 + 1)", "N")]
        b += ["    }"]
    else:
        b += geom("t0", "N")
    b += ["  }"]
    body: List[str] = []   # one tile (@T@), its buffer @S@, the next tile's buffer @O@
    if not RS_PIPE:
        # this tile's loads, then the next tile's run-form words: two round trips per tile (the
        # column stream, then the walk's aggregate inputs), fewer registers
        body += ["    rsC = rsN; reC = reN; tbC = tbN; gmC = gmN; grC = grN;"]
        body += [x.replace("@LIVE@", "") for x in issue]
        body += ["    if (@T@ + 1 < t1) {"]
        body += ["  " + x for x in geom("(@T@ + 1)", "N")]
        body += ["    }"]
    body += ["    const i64 rs = rsC, re = reC, tb0 = tbC; const u64 m_ = gmC | 1ull; "
             "const i64 q0 = (i64)grC;"]
    if tk is not None:
        # key run of a list entry, relative to the tile's first run (lrn_)
        body.append("    const i64 qb_ = __shfl(q0, 0, 64); const int qr_ = (int)(q0 - qb_);")
    body += ["    const i64 row0 = tb0 + 64 * ln;",
             "    const i64 lo_ = rs - row0, hi_ = re - row0;",
             "    const int alo = lo_ <= 0 ? 0 : (lo_ >= 64 ? 64 : (int)lo_);",
             "    const int ahi = hi_ <= 0 ? 0 : (hi_ >= 64 ? 64 : (int)hi_);",
             "    const u64 am = alo >= ahi ? 0ull : ((ahi == 64 ? ~0ull : ((1ull << ahi) - 1ull)) & "
             "~((1ull << alo) - 1ull));",
             "    const unsigned sh_ = (unsigned)(q0 & 31);",
             "    const u64 lw_ = (u64)tw0@S@_ | ((u64)tw1@S@_ << 32);",
             "    const u64 hw_ = (u64)tw2@S@_;",
             "    const u64 T_ = sh_ ? ((lw_ >> sh_) | (hw_ << (64 - sh_))) : lw_;",
             ]
    if RS_LUT:
        # row tags by nibble: rows 4i..4i+3 take their tags from a 5-run window of T (the run
        # covering row 4i-1, then the runs starting in the nibble) through a 512-entry LDS
        # table indexed by (nibble of run starts, window) - 16 fixed steps instead of a loop
        # over the group's run starts (~15 VALU per start, ~20-28 starts for the slowest lane)
        body += ["    u64 d_ = (u64)dlut_[((unsigned)m_ & 15u) | ((((unsigned)T_ << 1) & 31u) << 4)];",
                 "    unsigned P_ = (unsigned)__popc((unsigned)m_ & 15u);",
                 "    #pragma unroll",
                 "    for (int i_ = 1; i_ < 16; ++i_) {",
                 "      const unsigned mn_ = (unsigned)(m_ >> (4 * i_)) & 15u;",
                 "      const unsigned ix_ = mn_ | (((unsigned)(T_ >> (P_ - 1u)) & 31u) << 4);",
                 "      d_ |= (u64)dlut_[ix_] << (4 * i_);",
                 "      P_ += (unsigned)__popc(mn_);",
                 "    }",
                 "    d_ &= am;"]
    else:
        body += [
             # only the group's own runs' tags (popc(m) of them) decide whether any row is set
             "    const int nr_ = __popcll(m_);",
             "    const u64 Tm_ = nr_ >= 64 ? T_ : (T_ & ((1ull << nr_) - 1ull));",
             "    u64 c_ = T_ ^ (T_ << 1), d_ = 0ull, mm_ = (am && Tm_) ? m_ : 0ull;",
             "    while (mm_) { const u64 lb_ = mm_ & (0ull - mm_); if (c_ & 1ull) d_ |= lb_; "
             "c_ >>= 1; mm_ ^= lb_; }",
             "    d_ ^= d_ << 1; d_ ^= d_ << 2; d_ ^= d_ << 4; d_ ^= d_ << 8; d_ ^= d_ << 16; "
             "d_ ^= d_ << 32;",
             "    d_ &= am;"]
    if xpose:
        # the transpose slab and the passing-row list share the LDS: a tile's list is built
        # after its columns left the slab, and walked before the next tile's transpose
        lst_i = next(i for i, x in enumerate(b) if "__shared__ unsigned short lst_" in x)
        nslot = max(slab, (CAP * 2 + 15) // 16)
        # lst_[w] = wavefront w's own slab, seen as 16-bit entries
        b[lst_i:lst_i + 1] = [
            f"  __shared__ hs_v4u xt_[{WV}][{nslot}];",
            f"  unsigned short (*lst_)[{nslot * 8}] = (unsigned short (*)[{nslot * 8}])&xt_[0][0];"]
        body += xpose
    # predicate mask: 64 compares, shift-or into two 32-bit halves (a C loop: each row's
    # value is decoded where it is compared, not all 64 held decoded at once)
    body.append("    unsigned plo_ = 0u, phi_ = 0u;")
    cond = J._rename(g1.cnf(lpreds), pslots, "k")
    # narrow compact-code ranges: fail bits from a sign word (no compares, no constants held in
    # registers for the select), else the generic condition's pass bits
    sign = g1.cnf_sign(lpreds)
    if sign is not None:
        sign = J._rename(sign, pslots, "k")
    # two rows per 32-bit word (16-bit signed codes): packed saturating range tests, fail bits
    # gathered in even/odd order per 32-row half, then unzipped (2.5 VALU per row instead of 5)
    sign2 = g1.cnf_sign2(lpreds, "x{}w@S@[w_]") if RS_PK16 and sign is not None and \
        all(J._SIZEOF.get(g1.raw_type(sl)) == 2 for sl in pslots) else None
    if p12:
        # 12-bit chunks: decode 8 rows per 3 dwords, pair them into 16-bit halves, packed tests
        sign12 = g1.cnf_sign2(lpreds, "pw{}_", offset="a.P12O_{}")
        assert sign12 is not None
        for i in range(8):
            body.append("    {")
            for sl in p12:
                body += [f"      const unsigned a{sl}_ = x{sl}q@S@[{3 * i}], "
                         f"b{sl}_ = x{sl}q@S@[{3 * i + 1}], c{sl}_ = x{sl}q@S@[{3 * i + 2}];",
                         f"      const unsigned v{sl}_0 = a{sl}_ & 0xFFFu, "
                         f"v{sl}_1 = (a{sl}_ >> 12) & 0xFFFu, "
                         f"v{sl}_2 = ((a{sl}_ >> 24) | (b{sl}_ << 8)) & 0xFFFu, "
                         f"v{sl}_3 = (b{sl}_ >> 4) & 0xFFFu;",
                         f"      const unsigned v{sl}_4 = (b{sl}_ >> 16) & 0xFFFu, "
                         f"v{sl}_5 = ((b{sl}_ >> 28) | (c{sl}_ << 4)) & 0xFFFu, "
                         f"v{sl}_6 = (c{sl}_ >> 8) & 0xFFFu, v{sl}_7 = c{sl}_ >> 20;"]
            for q in range(4):
                w = 4 * i + q
                half, wl = ("plo_", w) if w < 16 else ("phi_", w - 16)
                body.append("      {")
                for sl in p12:
                    body.append(f"        const unsigned pw{sl}_ = v{sl}_{2 * q} | "
                                f"(v{sl}_{2 * q + 1} << 16);")
                body += [f"        const unsigned s2_ = {sign12};",
                         f"        {half} |= (s2_ >> {15 - wl}) & {(1 << wl) | (1 << (wl + 16))}u;",
                         "      }"]
            body.append("    }")
        body += ["    plo_ = hs_unzip16(plo_);", "    phi_ = hs_unzip16(phi_);"]
    elif sign2 is not None:
        for half, off in (("plo_", 0), ("phi_", 16)):
            body += ["    #pragma unroll",
                     "    for (int w_ = 0; w_ < 16; ++w_) {",
                     f"      const unsigned s2_ = {sign2.replace('[w_]', f'[w_ + {off}]')};",
                     f"      {half} |= (s2_ >> (15 - w_)) & ((1u << w_) | (1u << (w_ + 16)));",
                     "    }",
                     f"    {half} = hs_unzip16({half});"]
    for half, off in ((("plo_", 0), ("phi_", 32)) if sign2 is None and not p12 else ()):
        body.append("    #pragma unroll")
        body.append("    for (int k_ = 0; k_ < 32; ++k_) {")

        def raw_of(name: str) -> str:
            et, word, bits, per = elem[name]
            i = f"{off} + k_"
            w = word.format(i=i)
            return f"(({et})({w} >> ({bits} * (({i}) % {per}))))" if per > 1 else f"(({et}){w})"
        for sl in pslots:
            ct = J._CTYPE[cols[sl][0]]
            enc = cols[sl][2]
            raw = raw_of(f"x{sl}")
            body.append(f"      const auto xr{sl}_k = {raw};")
            raw = f"xr{sl}_k"
            if enc:
                body.append(f"      const int r{sl}_k = (int){raw};")
            if enc and enc[1]:
                bq = args.add("q", f"B{sl}", "long long")
                body.append(f"      const i64 q{sl}_k = {bq} + (i64){raw};")
            body.append(f"      const {ct} x{sl}_k = {g1.decode(sl, raw)};")
            if cols[sl][1]:
                body.append(f"      const bool n{sl}_k = {raw_of(f'n{sl}')} != 0;")
        if sign is not None:
            body.append(f"      {half} |= ((unsigned)({sign}) >> 31) << k_;")
        else:
            body.append(f"      {half} |= ({cond} ? 1u : 0u) << k_;")
        body.append("    }")
    if sign is not None:
        body += ["    d_ &= ~(((u64)phi_ << 32) | (u64)plo_);"]
    else:
        body += ["    d_ &= ((u64)phi_ << 32) | (u64)plo_;"]
    if RS_PIPE:
        # this tile's column words are consumed: the next tile's loads go out now
        # (the scheduler must not hoist the next tile's loads above this tile's masks: both
        # buffers would be live at once)
        # The loads are unconditional - a load under a condition keeps the buffer's previous
        # contents live through the whole tile - and past the wavefront's last tile they read
        # an empty buffer range (no memory traffic; the tag words re-read this tile's).
        body += ["    __builtin_amdgcn_sched_barrier(0);",
                 "    { const bool nx_ = @T@ + 1 < t1;",
                 "      if (nx_) { rsC = rsN; reC = reN; tbC = tbN; gmC = gmN; grC = grN; }"]
        body += ["  " + x.replace("@S@", "@O@").replace("@LIVE@", "!nx_ ? 0ll : ")
                 for x in issue]
        body += ["      if (@T@ + 2 < t1) {"]
        body += ["    " + x for x in geom("(@T@ + 2)", "N")]
        body += ["      }", "    }"]
    body += [
          # exclusive scan of the lanes' passing-row counts
          "    const int cn_ = __popcll(d_);",
          "    int inc_ = cn_;",
          "    for (int o_ = 1; o_ < 64; o_ <<= 1) { const int y_ = __shfl_up(inc_, o_, 64); "
          "if (ln >= o_) inc_ += y_; }",
          "    const int tot_ = __shfl(inc_, 63, 64);",
          f"    for (int wb_ = 0; wb_ < tot_; wb_ += {CAP}) {{",
          f"    const int wn_ = tot_ - wb_ < {CAP} ? tot_ - wb_ : {CAP};",
          "    { int pos_ = inc_ - cn_ - wb_; u64 e_ = d_;",
          "      while (e_) { const int bq_ = __builtin_ctzll(e_); "
          f"if (pos_ >= 0 && pos_ < {CAP}) {{ lst_[wq][pos_] = (unsigned short)(64 * ln + bq_); "
          + ("lrn_[wq][pos_] = (unsigned short)(qr_ + __popcll(m_ & ((2ull << bq_) - 1ull))); "
             if tk is not None else "") +
          "} ++pos_; e_ &= e_ - 1ull; } }",
          f"    {J._wave_sync()}",
          f"    for (int cb = 0; cb < wn_; cb += {64 * EW}) {{"]
    layout = pack_layout(p, compacts)
    if layout:
        body.append("      const u64* PKt_ = a.PK + tb0;")
    ind2 = "      "
    for k in range(EW):
        body += [f"{ind2}const int ce{k} = cb + {64 * k} + ln;",
                 f"{ind2}const bool cok{k} = ce{k} < wn_;",
                 f"{ind2}const int cof{k} = cok{k} ? (int)lst_[wq][ce{k}] : 0;",
                 f"{ind2}const i64 crow{k} = tb0 + (i64)cof{k};"]
        if tk is not None:
            body.append(f"{ind2}const unsigned crn{k} = cok{k} ? (unsigned)lrn_[wq][ce{k}] : "
                        f"0xFFFFFFFFu;")
    gs = [J._Gen(args, cols, SPLIT, (f"crow{k}", f"crow{k}"), approx, True) for k in range(EW)]
    packed = {sl: (off, nb) for sl, off, nb in layout} if layout else {}
    if layout:
        args.add("p", "PK", "const unsigned long long*")
    for k in range(EW):
        if layout:
            # the tile's rows through a uniform base: 32-bit lane offsets
            body.append(f"{ind2}const u64 pk{k}_ = PKt_[cof{k}];")
        for sl in tail:
            if sl in packed:
                off, nb = packed[sl]
                ct = gs[k].raw_type(sl)
                ut = {1: "unsigned char", 2: "unsigned short", 4: "unsigned"}[nb]
                J._uload_raw(gs[k], sl, f"c{k}", f"(({ct})({ut})(pk{k}_ >> {off}))", "1", body,
                             ind2)
            else:
                J._uload(gs[k], sl, f"c{k}", body, ind2)
    carry_gen = J._Gen(args, cols, SPLIT, ("tcw_", "tcw_"), frozenset(), True) \
        if tk is not None else None
    for k in range(EW):
        g = gs[k]
        it = f"c{k}"
        body.append(f"{ind2}{{ bool cok = cok{k};")
        gvar = "gic"
        if grouped:
            base = args.add("q", "group_base", "long long")
            ng = args.add("q", "num_groups", "long long")
            body.append(f"{ind2}const i64 glc = (i64){J._rename(f'x{p.group_col}', tail, it)} - "
                        f"{base};")
            body.append(f"{ind2}cok = cok && {J._rename(g.ok(p.group_col), tail, it)} && "
                        f"glc >= 0 && glc < {ng};")
            body.append(f"{ind2}const int {gvar} = cok ? (int)glc : 0;")
        if hk is not None:
            body += [J._rename(x, tail, it)
                     for x in JH._hash_accumulate(g, aggs, hk, "cok", ind2, tk=tk,
                                                 seg=f"crn{k}" if tk is not None else None,
                                                 row=f"crow{k}", run=f"qb_ + (i64)crn{k}",
                                                 carry_gen=carry_gen)]
        else:
            body += [J._rename(x, tail, it)
                     for x in J._accumulate(g, aggs, grouped, "cok", gvar, ind2)]
        body.append(f"{ind2}}}")
    body += ["    }", f"    {J._wave_sync()}", "    }"]

    def tile(tv: str, cur: str, nxt: str) -> List[str]:
        return ["   {"] + [x.replace("@T@", tv).replace("@S@", cur).replace("@O@", nxt)
                          for x in body] + ["   }"]
    if RS_PIPE == 2:
        b += ["  for (i64 t = t0; t < t1; t += 2) {"]
        b += tile("t", "A", "B")
        b += ["    if (t + 1 >= t1) break;"]
        b += tile("(t + 1)", "B", "A")
        b += ["  }"]
    elif RS_PIPE:
        b += ["  for (i64 t = t0; t < t1; ++t) {"]
        b += tile("t", "A", "A")
        b += ["  }"]
    else:
        b += ["  for (i64 t = t0; t < t1; ++t) {"]
        b += tile("t", "A", "A")
        b += ["  }"]
    if hk is None:
        b += J._flush(aggs, grouped)
    if tk is not None:
        b += JH._topk_carry_final(aggs, hk, tk, "  ", carry_gen)

        def key_lines(j: int, ind_: str) -> List[str]:
            gk = J._Gen(args, cols, SPLIT, (f"tkr{j}", f"tkr{j}"), frozenset(), True)
            out: List[str] = []
            for c in hk.cols:
                J._uload(gk, c.slot, "F", out, ind_)
            out += JH._hash_key_lines(gk, hk, "tkey_l", "_F", ind_)
            out.append(f"{ind_}const u64 tkey_ = tkey_l;")
            return out
        b += JH._topk_flush(aggs, tk, args, "wid", key_lines)
    name = "hs_jit_run_bits_scan" if hk is None else \
        ("hs_jit_run_bits_hash" if tk is None else "hs_jit_run_bits_topk")
    occ = f" __attribute__((amdgpu_waves_per_eu({RS_WAVES}, {RS_WAVES})))" if RS_WAVES else ""
    src = (J._PRELUDE + args.struct_src() +
           f'extern "C" __global__ __launch_bounds__({BLOCK}){occ} void {name}(Args a) '
           f'{{\n' + "\n".join(b) + "\n}\n")
    lds = (len(aggs) * p.num_groups * 32) if grouped else 0
    return J.Kernel(src, name, args, lds)


class TwoPhaseLauncher:
    """Both phases lowered once (kernels, tiles, spans, per-tile run windows, the tag bitmap);
    ``launch(p)`` fills the literal slots and queues: bitmap clear, tags, scan, partials fold."""
    __slots__ = ("kt", "ks", "grid_t", "grid_s", "GA", "shmem", "vt", "vs", "compacts", "keep",
                 "tags", "dev", "blocks", "hk", "graph", "gblocks", "tk", "tpl", "match",
                 "launches")

    def __init__(self, kt, ks, grid_t, grid_s, GA, shmem, vt, vs, compacts, keep, tags, dev,
                 hk=None, tk=None):
        self.kt, self.ks, self.grid_t, self.grid_s = kt, ks, grid_t, grid_s
        self.GA, self.shmem, self.vt, self.vs = GA, shmem, vt, vs
        self.compacts, self.keep, self.tags, self.dev = compacts, keep, tags, dev
        # literal vector -> (phase-1 block, phase-2 block template): a repeated parameter set
        # re-packs only the per-launch partials pointers
        self.blocks: dict = {}
        # hash-mode phase 2 (a KeyPlan): groups go to a device hash table, no partials
        self.hk = hk
        self.tk = tk          # run top-K mode of the hash walk (hash_agg.TopKPlan)
        # the captured pipeline (graphs.TwoPhaseGraph) and its per-literal-vector blocks
        self.graph = None
        self.gblocks: dict = {}
        # packed argument blocks of the literal-independent slots: a new literal vector patches
        # only its literal slots into copies of these
        self.tpl = None
        # (W, runs, lowered parameters) while phase 1 may still switch to a recorded match
        # (RT2_MATCH): on the launcher's second launch - a lowering that is reused - ``_record``
        self.match = None
        self.launches = 0

    def _record(self) -> None:
        """Switch phase 1 to the recorded-match form: one verifying launch stores each run's
        right row (``record_matches``), later launches read it.  Skipped when the record would
        not fit the device's free memory with a margin; the record counts against the table
        caches' budgets while it lives (``device_cache.track_derived``)."""
        import torch
        from .device_cache import track_derived
        W, nruns, p = self.match
        self.match = None
        need = ((nruns + 63) >> 6) * 64 * 16
        free, _ = torch.cuda.mem_get_info(self.dev)
        free += torch.cuda.memory_reserved(self.dev) - torch.cuda.memory_allocated(self.dev)
        if free < need + (8 << 30):
            return
        try:
            m = record_matches(p, self.compacts, W, self.vt, nruns, self.grid_t, self.dev)
            mode = "copy" if RT2_COPY and copy_ok(p, self.compacts) else "match"
            if mode == "copy":
                held, vals = copy_matches(p, self.compacts, m, self.vt, self.dev)
                # (the match record itself is dropped once the gather ran: stream-ordered frees)
            else:
                held, vals = [m], {"MATCH": m.data_ptr()}
        except torch.OutOfMemoryError:
            return      # an optional copy: the verifying form stays
        for t in held:
            track_derived(t)
        self.kt = J.kernel_for(tags2_shape(p, self.compacts, W, True, mode),
                               lambda: gen_run_tags2(p, self.compacts, W, True, mode))
        self.vt = dict(self.vt, **vals)
        self.keep = self.keep + tuple(held)
        # every packed phase-1 block and the captured pipeline name the verifying kernel
        self.tpl, self.graph = None, None
        self.blocks.clear()
        self.gblocks.clear()

    def graphable(self) -> bool:
        """Whether one query's launches can be captured: partials out (not the hash mode)."""
        return self.hk is None

    def launch(self, p: NL.JoinParams, key=None, htab=None, hk=None, graph: bool = False):
        """Queue one query.  Returns the (sum, count, min, max) device outputs, or with
        ``graph`` (and a literal vector ``key``) a ``graphs.GraphPending`` of one replay of the
        captured pipeline."""
        import struct
        self.launches += 1
        if self.match is not None and self.launches == 2:
            self._record()
        st = NL.stream_ptr()
        if self.hk is not None:
            preds = [(k_, p.preds[k_]) for k_ in range(p.npreds)]
            vt = dict(self.vt)
            J.fill_preds_aggs(vt, preds, [], self.compacts)
            vs = dict(self.vs)
            vs.update({"psum": 0, "pcnt": 0, "pmin": 0, "pmax": 0})
            J.fill_preds_aggs(vs, preds, [p.aggs[i] for i in range(p.naggs)], self.compacts)
            vs.update(htab.kernel_values())
            vs.update((hk or self.hk).values())   # this query's key domain
            if self.tk is not None:
                vs.update(self.tk.kernel_values())
                self.tk.used = True
            self.kt.launch(self.grid_t, vt, st, 0)
            self.ks.launch(self.grid_s, vs, st, self.shmem)
            if self.tk is not None:
                self.tk.finish(st)
            return None
        hit = self.blocks.get(key) if key is not None else None
        if hit is None:
            preds = [(k_, p.preds[k_]) for k_ in range(p.npreds)]
            aggs = [p.aggs[i] for i in range(p.naggs)]
            if self.tpl is None:
                vs0 = dict(self.vs)
                vs0.update({"psum": 0, "pcnt": 0, "pmin": 0, "pmax": 0})
                self.tpl = (bytes(self.kt.args.pack(self.vt, default=0)),
                            bytes(self.ks.args.pack(vs0, default=0)))
            lt: dict = {}
            J.fill_preds_aggs(lt, preds, [], self.compacts)
            ls: dict = {}
            J.fill_preds_aggs(ls, preds, aggs, self.compacts)
            hit = (bytes(self.kt.args.patch(bytearray(self.tpl[0]), lt)),
                   self.ks.args.patch(bytearray(self.tpl[1]), ls))
            if key is not None:
                if len(self.blocks) >= 256:
                    self.blocks.clear()
                self.blocks[key] = hit
        if graph and key is not None and self.graphable():
            from .graphs import GraphPending, TwoPhaseGraph, _cbuf
            g = self.graph
            if g is None:
                g = self.graph = TwoPhaseGraph(self.kt, self.ks, self.grid_t, self.grid_s,
                                               self.GA, self.shmem, self.dev)
            gb = self.gblocks.get(key)
            if gb is None:
                bs = bytearray(hit[1])
                a = self.ks.args
                for name, ptr in g.partial_ptrs().items():
                    struct.pack_into("<q", bs, a.offset(name), ptr)
                gb = (_cbuf(hit[0]), _cbuf(bs))
                if len(self.gblocks) >= 256:
                    self.gblocks.clear()
                self.gblocks[key] = gb
            return GraphPending(g, g.launch(*gb))
        # (phase 1 stores every word of every run group: no bitmap clear)
        self.kt.launch_packed(self.grid_t, hit[0], st)
        parts = J._partials(self.grid_s, self.GA, self.dev)
        bs = bytearray(hit[1])
        a = self.ks.args
        for name, t in zip(("psum", "pcnt", "pmin", "pmax"), parts):
            struct.pack_into("<q", bs, a.offset(name), t.data_ptr())
        self.ks.launch_packed(self.grid_s, bs, st, self.shmem)
        return J._final(parts, self.grid_s, self.GA, self.dev)


def lower(p: NL.JoinParams, rstart, rlen, rbucket, roff, compacts, runs, nrows: int,
          cache_spans: bool, hk=None, tk=None, record: bool = False) -> Optional[TwoPhaseLauncher]:
    """The two-phase launcher of a run-keyed merge join, or None when it does not apply.
    ``hk``: group by that hash key plan (left-side key columns only) through the bits scan's
    hash mode (needs 1-bit tags).  None for an empty right side too (nothing to match)."""
    import torch
    if not applies(p) or runs is None or int(roff[-1].item()) <= 0:
        return None
    if hk is not None and (not RS_BITS or tag_width(p) != 1 or _scan_grouped(p) or
                           any(s >= SPLIT for s in hk.slots)):
        return None
    W = tag_width(p)
    NI = RS_ITEMS if RS_ITEMS and 64 % RS_ITEMS == 0 else J._mj_items(True)
    T = J.BLOCK * NI  # noqa: N806
    dev = rstart.device
    max_tiles = nrows // T + 2 * rstart.numel() + 2
    tp, spans = J._join_spans(p, rstart, rlen, rbucket, roff, max_tiles, T, cache_spans, align=NI)
    onebit = W == 1 and not (_scan_grouped(p) and p.group_col >= SPLIT)
    sparse = RS_BITS and onebit
    if tk is not None and hk is None:
        tk = None
    if sparse:
        ks = J.kernel_for(sparse_shape(p, compacts, hk, tk),
                          lambda: gen_run_sparse_scan(p, compacts, hk, tk))
    else:
        ks = J.kernel_for(scan_shape(p, compacts, W, NI),
                          lambda: gen_run_scan(p, compacts, W, NI))
    nruns = int(runs.runkeys.numel())
    KW = ((31 + (NI - 1) * W) >> 5) + 1  # noqa: N806
    nwords = max((nruns * W + 31) >> 5, ((nruns + 63) >> 6) * 2 * W)
    tags = torch.empty(nwords + KW + 2, dtype=torch.int32, device=dev)
    frame = J._key32_frame(p, compacts)
    rng = run_ranges(rstart, rlen, rbucket, roff, runs)
    rng_d = torch.from_numpy(rng.reshape(-1).copy() if len(rng) else
                             __import__("numpy").zeros(4, "int64")).to(dev)
    # 32-bit run / right-row indices when both fit (with slack for the gallop's overshoot)
    ix32 = RT2_I32 and nruns < (1 << 31) - (1 << 20) and int(roff[-1].item()) < (1 << 31) - (1 << 20)
    kt = J.kernel_for(tags2_shape(p, compacts, W, ix32),
                      lambda: gen_run_tags2(p, compacts, W, ix32))
    vt = {"RNG": rng_d.data_ptr(), "NRG": len(rng), "NRUNS": nruns, "tags": tags.data_ptr(),
          "num_groups": p.num_groups, "group_base": p.group_base}
    tr = rng_d
    grid_t = max(1, RT2_GRID)
    vt["KLO"], vt["KSP"], vt["KOF"] = frame
    J._fill_cols(vt, p.cols, compacts)
    lo = lo16_keys(p, compacts, W, vt, nruns, int(roff[-1].item()), grid_t, dev) \
        if RT2_LO16 and ix32 and cache_spans else None
    if lo is not None:
        kt = J.kernel_for(tags2_shape(p, compacts, W, ix32, "lo16"),
                          lambda: gen_run_tags2(p, compacts, W, ix32, "lo16"))
        vt["LL"], vt["RL"] = lo[0].data_ptr(), lo[1].data_ptr()
        tr = (rng_d, lo)
    vs = {"rstart": rstart.data_ptr(), "rlen": rlen.data_ptr(), "tile_prefix": tp.data_ptr(),
          "tags": tags.data_ptr(), "R": rstart.numel(), "nrows": nrows,
          "num_groups": p.num_groups, "group_base": p.group_base}
    J._fill_cols(vs, p.cols, compacts)
    GA = p.naggs * (p.num_groups if p.group_col >= 0 else 1)
    grid_s = max(1, J.SCAN_GRID or NL.lib().hs_scan_grid())
    if sparse:
        from ..ops import kernels as K
        tp64 = K.ranges_to_tiles(rlen + (rstart & 63), 4096)   # 64-aligned 4096-row tiles
        vs["tile_prefix"] = tp64.data_ptr()
        layout = pack_layout(p, compacts)
        pk = packed_tail(layout, compacts) if layout else None
        if pk is not None:
            vs["PK"] = pk.data_ptr()
        spans = (spans, tp64, pk, fill_pack12(vs, p, compacts))
        grid_s = max(1, RS_BITS_GRID)
    if tk is not None:
        tk.bind(grid_s * (J.BLOCK // 64), dev)
    lz = TwoPhaseLauncher(kt, ks, grid_t, grid_s, GA, GA * 32 if _scan_grouped(p) else 0,
                          vt, vs, compacts, (rstart, rlen, rbucket, roff, tp, spans, tr, runs),
                          tags, dev, hk, tk if sparse else None)
    if record and RT2_MATCH and ix32:
        # the lowering's own parameters: a later launch's may bind other column slots
        lz.match = (W, nruns, NL.JoinParams.from_buffer_copy(p))
    return lz


def semi_runs_agg(p: NL.JoinParams, rstart, rlen, compacts, runs, nrows: int, words, lo: int,
                  nbits: int):
    """A semi-join probe (``attr in <build-key bitmap>``, GpuBackend._semi_join_agg) over the
    probe key's run form: one bitmap test per run (``hs_run_bitmap_tags``: 1-bit run tags), then
    the bit-parallel phase 2 (``gen_run_sparse_scan``) with the probe's own predicates and
    aggregates - the per-row key read and bitmap test of the plain scan become per-run.  ``p``
    carries the probe side only (slots < SPLIT, ``p.lkey`` = the key slot, ``p.nlp ==
    p.npreds``).  Returns the aggregate outputs (sums, counts, mins, maxs)."""
    import torch
    from ..ops import kernels as K
    dev = rstart.device
    nruns = int(runs.runkeys.numel())
    G = (nruns + 63) >> 6  # noqa: N806
    tags = torch.empty(2 * G + 4, dtype=torch.int32, device=dev)
    st = NL.stream_ptr()
    NL.check(NL.lib().hs_run_bitmap_tags(runs.runkeys.data_ptr(), nruns, int(runs.base) - int(lo),
                                         words.data_ptr(), int(nbits), tags.data_ptr(), st),
             "hs_run_bitmap_tags")
    ks = J.kernel_for(sparse_shape(p, compacts), lambda: gen_run_sparse_scan(p, compacts))
    tp64 = K.ranges_to_tiles(rlen + (rstart & 63), 4096)
    vs = {"rstart": rstart.data_ptr(), "rlen": rlen.data_ptr(), "tile_prefix": tp64.data_ptr(),
          "tags": tags.data_ptr(), "R": rstart.numel(), "nrows": nrows,
          "num_groups": p.num_groups, "group_base": p.group_base}
    J._fill_cols(vs, p.cols, compacts)
    layout = pack_layout(p, compacts)
    pk = packed_tail(layout, compacts) if layout else None
    if pk is not None:
        vs["PK"] = pk.data_ptr()
    p12 = fill_pack12(vs, p, compacts)
    GA = p.naggs * (p.num_groups if p.group_col >= 0 else 1)  # noqa: N806
    grid = max(1, RS_BITS_GRID)
    parts = J._partials(grid, GA, dev)
    vs.update({"psum": parts[0].data_ptr(), "pcnt": parts[1].data_ptr(),
               "pmin": parts[2].data_ptr(), "pmax": parts[3].data_ptr()})
    J.fill_preds_aggs(vs, [(k_, p.preds[k_]) for k_ in range(p.npreds)],
                      [p.aggs[i] for i in range(p.naggs)], compacts)
    ks.launch(grid, vs, st, GA * 32 if _scan_grouped(p) else 0)
    out = J._final(parts, grid, GA, dev)
    for t in (tags, tp64, pk, *p12):   # used by the queued kernels: keep until they ran
        if t is not None:
            t.record_stream(torch.cuda.current_stream(dev))
    return out
