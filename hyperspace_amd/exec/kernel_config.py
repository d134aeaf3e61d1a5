"""Code-generation tunables of the generated HIP kernels, as ONE frozen configuration.

Every knob the kernel generators (``exec/jit.py``, ``exec/jit_runs.py``) read is a field here,
with its measured default.  A configuration is built once - from the session conf
(``spark.hyperspace.mi.kernel.<field>``, e.g. ``spark.hyperspace.mi.kernel.mj_grid``) over the
``HS_JIT_<FIELD>`` environment (sweep scripts) over the defaults - and bound into the generators'
module constants by ``bind``; kernel shape keys include those constants, so a different
configuration never reuses another's compiled kernels.  The binding is process-wide (the
generated-kernel cache is too): ``GpuBackend`` binds its session's configuration when it comes
up, and tests and sweeps switch configurations with ``use(...)``, which restores the previous
one - nothing assigns the generators' module globals directly.

Fields marked "alternative" are measured variants kept because a test exercises them (their
records are in ``profiles/``); variants that lost and had no remaining use were deleted.
"""
from __future__ import annotations

import contextlib
import dataclasses
import os
import threading
from typing import Dict, Iterator

CONF_PREFIX = "spark.hyperspace.mi.kernel."
ENV_PREFIX = "HS_JIT_"


@dataclasses.dataclass(frozen=True)
class KernelConfig:
    # --- scan kernel (gen_scan_agg) ---------------------------------------------------------
    scan_items: int = 4          # rows per thread of the strided scan
    scan_grid: int = 8192        # scan grid (blocks)
    scan_vec: int = 8            # rows per thread of the vectorized scan (aligned vector loads)
    scan_compact: bool = True    # aggregate inputs loaded for passing rows only (LDS lists)
    scan_eager: bool = False     # alternative: every column in the first batch
    # --- generic join kernel (gen_join_agg); 512-row tiles on a 16384-block grid measured best
    # (profiles/microbench_join_r1*.jsonl) ------------------------------------------------------
    join_items: int = 2
    join_block: int = 256
    join_lds_keys: int = 2048
    join_grid: int = 16384
    join_eager: bool = False     # alternative (lazy loads won, profiles/microbench_join_r1c)
    join_stage_right: bool = True
    join_pipeline: bool = True   # next tile's batch loads overlap this tile's work
    join_direct: bool = False    # alternative: direct-address LDS key table (5.18 vs 3.98 ms)
    join_direct_slots: int = 2048
    # --- join-index kernel (gen_join_index_agg) ---------------------------------------------
    ji_items: int = 4
    ji_vec: int = 8
    ji_compact: bool = True
    ji_stage: bool = False       # alternative: LDS copy of the matched right rows
    ji_bitmap: bool = False      # alternative: right predicates as a per-row bitmap
    # --- single-kernel sort-merge join (gen_merge_join_agg) ---------------------------------
    mj_items: int = 8
    mj_lds_keys: int = 2048
    mj_grid: int = 8192
    mj_steps: int = 1            # branch-free walk steps per row
    mj_stage_unroll: int = 4     # right-span staging rows per thread per round trip
    mj_block: int = 256
    mj_dbuf: bool = False        # alternative: double-buffered LDS spans
    mj_prefetch: bool = False    # alternative: next tile's span prefetch
    mj_rpf: bool = False         # alternative: span bounds prefetch (1.63 vs 1.40 ms)
    mj_eager: bool = False       # alternative: eager aggregate tail
    mj_sparse: bool = True       # match-list appends one set bit per round
    mj_hash_lanemajor: bool = False  # alternative: hash-mode matches appended lane-major
    mj_key32: bool = True        # 32-bit merge images
    mj_key16: bool = False       # alternative: grouped 16-bit left keys (1.51 vs 1.38 ms)
    mj_runs: bool = True         # run-keyed merge join over a left key's run-length form
    mj_runs_hash: bool = True    # hash-mode GROUP BY over the two-phase run walk
    mj_runs_items: int = 16
    mj_runs_prefetch: bool = False   # alternative
    # --- two-phase run-keyed join (exec/jit_runs.py) ----------------------------------------
    mj_2p: bool = True           # two phases (tags, then the left rows' scan)
    rs_items: int = 16           # rows per thread of the dense phase-2 scan (W > 1 tags)
    rt2_unroll: int = 4          # phase-1 64-run groups in flight per wavefront iteration
    rt2_grid: int = 8192
    rt2_i32: bool = True         # phase-1 run / right-row index math in 32 bits when tables fit
    rt2_match: bool = True       # phase 1 reads a per-run matched right row recorded at lowering
    #                              (literal-independent) instead of re-verifying the key match
    rt2_copy: bool = True        # ... and the right predicate / group columns gathered into run
    #                              order with it (one hit bit per run): nothing read at right rows
    rt2_lo16: bool = False       # phase 1 compares 16-bit key halves in groups whose end keys
    #                              matched in full with a key span < 2^16 (reused lowerings):
    #                              correct, but 303 -> 465 us at SF100 (profiles/tags2_lo16_r6.txt)
    rs_bits: bool = True         # phase 2 bit-parallel for 1-bit tags (gen_run_sparse_scan)
    rs_bits_grid: int = 8192
    rs_pack: bool = True         # bits scan reads its aggregate inputs row-packed
    rs_pipe: int = 0             # bits scan software pipeline: 0 off (two round trips per tile,
                                 # fewest registers), 1 one buffer, 2 two named buffers (unroll 2);
                                 # SF100: 358 / 363 / 391 us (profiles/bits_scan_variants_r6.txt)
    rs_walk: int = 4             # bits scan list entries per lane per walk pass
    rs_pk16: bool = True         # bits scan range tests of 16-bit codes two rows per packed op
    rs_waves: int = 0            # bits scan waves per SIMD the compiler must fit (0: its choice)
    rs_pack12: bool = True       # bits scan reads 16-bit predicate codes within [0, 4095] from a
                                 # 12-bit packed copy (25% fewer bytes of its row stream)
    rs_lut: bool = True          # bits scan row tags by nibble through an LDS table (else a loop
                                 # over each group's run starts + prefix XOR)
    rs_lds: bool = False         # bits scan predicate columns loaded lane-coalesced, then moved
                                 # to their rows' lanes through LDS (else one 128 B run per lane)
    # --- shared ------------------------------------------------------------------------------
    vec_prefetch: bool = True    # software-pipelined full tiles of the vectorized kernels
    wave_sync: bool = True       # per-wavefront lists ordered by a wavefront barrier

    # -- construction ------------------------------------------------------------------------
    @staticmethod
    def _parse(f: dataclasses.Field, raw) -> object:
        if f.type in (bool, "bool"):
            return str(raw).strip().lower() in ("1", "true", "yes", "on")
        return int(raw)

    @classmethod
    def from_env(cls, env=None) -> "KernelConfig":
        """Defaults overridden by ``HS_JIT_<FIELD>`` variables (sweeps and microbenchmarks)."""
        env = os.environ if env is None else env
        kw = {}
        for f in dataclasses.fields(cls):
            raw = env.get(ENV_PREFIX + f.name.upper())
            if raw is not None and raw != "":
                kw[f.name] = cls._parse(f, raw)
        return cls(**kw)

    def with_conf(self, conf) -> "KernelConfig":
        """This configuration overridden by ``spark.hyperspace.mi.kernel.<field>`` keys."""
        kw = {}
        for f in dataclasses.fields(self):
            raw = conf.get(CONF_PREFIX + f.name, None)
            if raw is not None and raw != "":
                kw[f.name] = self._parse(f, raw)
        return dataclasses.replace(self, **kw) if kw else self

    def replace(self, **kw) -> "KernelConfig":
        return dataclasses.replace(self, **kw)

    def as_dict(self) -> Dict[str, object]:
        return dataclasses.asdict(self)


_BASE = KernelConfig.from_env()
_active = _BASE
_lock = threading.RLock()


def active() -> KernelConfig:
    return _active


def base() -> KernelConfig:
    """The process's configuration before any session conf (defaults + environment)."""
    return _BASE


def bind(cfg: KernelConfig) -> None:
    """Make ``cfg`` the generators' configuration: their module constants (upper-case field
    names) are set from it.  Compiled kernels are keyed by shape tuples that include those
    constants, so switching needs no cache flush for correctness."""
    global _active
    from . import jit, jit_join, jit_runs
    with _lock:
        for name, v in dataclasses.asdict(cfg).items():
            up = name.upper()
            for mod in (jit, jit_runs):
                if up in mod.__dict__:
                    setattr(mod, up, v)
        if cfg != _active:
            # lowerings cached by query shape hold the previous configuration's kernels
            jit_join._RUNS_LOWERED.clear()
            jit_join._RUNS_HASH_LOWERED.clear()
        _active = cfg


@contextlib.contextmanager
def use(cfg: KernelConfig = None, **overrides) -> Iterator[KernelConfig]:
    """``with kernel_config.use(mj_lds_keys=32): ...`` - a configuration for the block (tests,
    sweeps), restored afterwards."""
    with _lock:
        prev = _active
        new = (cfg or prev).replace(**overrides) if overrides else (cfg or prev)
        bind(new)
    try:
        yield new
    finally:
        bind(prev)


__all__ = ["KernelConfig", "active", "base", "bind", "use", "CONF_PREFIX"]
