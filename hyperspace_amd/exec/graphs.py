"""hipGraph-captured scan pipelines (BASELINE.json north star; SURVEY.md §2.3 K7 "kernel chain
captured in a hipGraph", §7.4 item 6).

An indexed filter + aggregate (TPC-H Q6 shape) is five device steps on the device-resident index
table:

1. per-bucket range search of the leading indexed column (``hs_range_search_dev``);
2. ranges -> tile prefix (``hs_ranges_to_tiles``);
3. the query's generated scan kernel (``exec/jit.py``);
4. the deterministic final reduction (``hs_agg_final``);
5. the D2H copy of the result block.

Every size in that chain is fixed by the table (one range per bucket, a fixed grid), so it is
captured ONCE per (query shape, table) into a HIP graph.  The graph's only input is a pinned
parameter block: the range bounds plus the generated kernel's argument block (its literals),
which the kernel reads through a device pointer.  A query of a known shape writes the block and
replays the graph: one launch instead of five, and none of the per-kernel host work.

The first execution of a key runs the same sequence eagerly (that also loads the kernel module)
and then captures; later executions replay.  With several ranks (sharded placement) the
replay's device output block is all-gathered across ranks right after it (exec/gpu.py); the
graph's own D2H then only feeds single-rank callers.
"""
from __future__ import annotations

import ctypes as C
import struct
import threading
from collections import OrderedDict
from typing import Optional, Tuple

import numpy as np

from ..ops import _lib as NL
from . import jit

PARAM_HEAD = 64   # 6 x int64 range bounds, padded to a cache line


class _Pinned:
    """A hipHostMalloc block (capture-safe: no allocator bookkeeping on the copies)."""

    def __init__(self, nbytes: int):
        self.nbytes = nbytes
        self.ptr = jit.runtime().hs_host_alloc(nbytes)
        if not self.ptr:
            raise MemoryError(f"hipHostMalloc({nbytes}) failed")

    def view(self) -> np.ndarray:
        v = getattr(self, "_view", None)
        if v is None:       # the block never moves: one numpy view for its lifetime
            v = self._view = np.ctypeslib.as_array((C.c_uint8 * self.nbytes).from_address(self.ptr))
        return v

    def __del__(self):
        if getattr(self, "ptr", None):
            jit.runtime().hs_host_free(self.ptr)
            self.ptr = None


class _Slot:
    """One in-flight instance of a captured pipeline: its own pinned parameter and result
    blocks (the graph's H2D reads the first and its D2H writes the second when the graph
    EXECUTES, so a query queued behind another must not share them), its own executable graph
    (whose kernel arguments are rewritten per launch), and the event that marks its result
    ready."""

    def __init__(self, params_bytes: int, out_bytes: int):
        self.h_params = _Pinned(max(params_bytes, 8))
        self.h_out = _Pinned(out_bytes)
        self.graph = None          # native handle (csrc/runtime/hs_graph.cpp)
        # native timing-disabled event: recorded by hs_graph_replay in the same call as the
        # launch (a torch.cuda.Event costs a few Python-level calls per query)
        self.event = jit.runtime().hs_event_create()
        if not self.event:
            raise RuntimeError(f"hs_event_create: {jit.runtime().hs_graph_last_error().decode()}")
        self.launched = False
        self.current = None   # _Launch whose result the slot's h_out holds / will hold

    def done(self) -> bool:
        rc = jit.runtime().hs_event_query(self.event)
        _rt_check(rc if rc < 0 else 0, "hs_event_query")
        return rc == 0

    def wait(self) -> None:
        _rt_check(jit.runtime().hs_event_sync(self.event), "hs_event_sync")

    def __del__(self):
        R = jit.runtime()
        if getattr(self, "graph", None):
            R.hs_graph_destroy(self.graph)
            self.graph = None
        if getattr(self, "event", None):
            R.hs_event_destroy(self.event)
            self.event = None


class _Launch:
    """One query launched into a slot; ``value`` is filled when it is read (by the caller, or
    by the next launch that needs the slot first)."""

    __slots__ = ("slot", "value")

    def __init__(self, slot: _Slot):
        self.slot = slot
        self.value = None


def _rt_check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what}: {jit.runtime().hs_graph_last_error().decode()}")


class _RingGraph:
    """A captured pipeline with ``RING`` in-flight instances (one pinned parameter block, one
    pinned result block and one executable graph per slot; device intermediates shared, since
    replays on one stream execute in order).  Subclasses define ``kernels`` (the generated
    kernels whose by-value argument blocks change per query), ``_enqueue(slot, stream, blocks)``
    (the work one query queues, eager or under capture), ``GA`` and ``out`` (the device result
    block, ``K.agg_outputs``).

    A replay rewrites the captured kernel nodes' argument blocks (``hs_graph_set_args``) and
    launches the executable graph: the kernels keep their by-value kernarg struct (a struct read
    from device memory makes every column load a flat load, ~2x slower on gfx950 -
    ``profiles/graph_byptr_r5.txt``)."""
    # in-flight instances per captured shape: a pipelined query stream (exec/gpu.py
    # collect_async) keeps a few replays of the same shape queued at once
    RING = 4

    def _init_ring(self, params_bytes: int) -> None:
        self.slots = [_Slot(params_bytes, self.out[0].hs_buf.numel()) for _ in range(self.RING)]
        self._next = 0
        self._warm = False
        self.replays = 0
        self.on_side = False   # replays moved to the backend's side stream (exec/gpu.py)
        self.side_stream = None

    @property
    def graph(self):
        return self.slots[0].graph

    def _capture(self, slot: _Slot, blocks, cur) -> None:
        import torch
        R = jit.runtime()
        side = torch.cuda.Stream()
        side.wait_stream(cur)
        _rt_check(R.hs_graph_capture_begin(side.cuda_stream), "hs_graph_capture_begin")
        try:
            self._enqueue(slot, side.cuda_stream, blocks)
        finally:
            fns = [k.function() for k in self.kernels]
            arr = (C.c_void_p * len(fns))(*fns)
            h = R.hs_graph_capture_end(side.cuda_stream, arr, len(fns))
        if not h:
            raise RuntimeError(f"graph capture: {R.hs_graph_last_error().decode()}")
        cur.wait_stream(side)
        slot.graph = h

    def _launch_slot(self, fill, blocks, stream=None, after=None) -> _Launch:
        """Queue one query on ``stream`` (default: the current stream), ordered after the work
        queued on ``after`` when given: ``fill(host_params)`` writes its pinned parameter block
        (a ``_Pinned``), ``blocks`` are the packed argument blocks (``_cbuf``) of ``kernels``.
        A slot still holding an unread earlier result is drained first (wait for it and keep
        its result on the earlier handle: back-pressure, no lost results); a slot's graph gets
        new kernel arguments only once its previous replay has finished.  A replay is one native
        call (``hs_graph_replay``: ordering, argument rewrite, launch, completion event)."""
        import torch
        slot = self.slots[self._next]
        self._next = (self._next + 1) % len(self.slots)
        prev = slot.current
        if prev is not None and prev.value is None:
            prev.value = self._read(slot)
        elif slot.launched and not slot.done():
            slot.wait()    # back-pressure: the slot's replay is still running
        fill(slot.h_params)
        R = jit.runtime()
        if slot.graph is not None:
            st = stream.cuda_stream if stream is not None else NL.raw_stream()
            ptrs = (C.c_void_p * len(blocks))(*[C.addressof(b) for b in blocks])
            _rt_check(R.hs_graph_replay(slot.graph, len(blocks), ptrs, st,
                                        after.cuda_stream if after is not None else None,
                                        slot.event), "hs_graph_replay")
            self.replays += 1
        else:
            cur = stream if stream is not None else torch.cuda.current_stream()
            st = cur.cuda_stream
            if after is not None:
                cur.wait_stream(after)
            if not self._warm:
                self._enqueue(slot, st, blocks)   # first run of the shape: eager (loads modules)
                self._warm = True
            else:
                self._capture(slot, blocks, cur)
                _rt_check(R.hs_graph_launch(slot.graph, st), "hs_graph_launch")
                self.replays += 1
            _rt_check(R.hs_event_record(slot.event, st), "hs_event_record")
        slot.launched = True
        h = _Launch(slot)
        slot.current = h
        return h

    def result(self, h: _Launch):
        """(sum, count, min, max) numpy arrays of the launched query ``h``."""
        if h.value is None:
            h.value = self._read(h.slot)
        return h.value

    def _read(self, slot: _Slot):
        slot.wait()
        h = slot.h_out.view()
        n = 8 * self.GA
        return (h[0:n].view(np.float64).copy(), h[n:2 * n].view(np.int64).copy(),
                h[2 * n:3 * n].view(np.float64).copy(), h[3 * n:4 * n].view(np.float64).copy())

    def _final_and_d2h(self, slot: _Slot, stream: int, grid: int) -> None:
        L = jit.runtime()
        K = NL.lib()
        p = self.parts
        o = self.out
        NL.check(K.hs_agg_final(NL.ptr(p[0]), NL.ptr(p[1]), NL.ptr(p[2]), NL.ptr(p[3]),
                                grid, self.GA, NL.ptr(o[0]), NL.ptr(o[1]), NL.ptr(o[2]),
                                NL.ptr(o[3]), stream), "hs_agg_final")
        NL.check(L.hs_memcpy_async(slot.h_out.ptr, o[0].hs_buf.data_ptr(), slot.h_out.nbytes, 2,
                                   stream), "result D2H")


def _cbuf(block) -> "C.Array":
    """A ctypes copy of a packed argument block (kept with the cached block, so a replay passes
    its address without a per-query copy)."""
    b = bytes(block)
    return C.create_string_buffer(b, len(b))


class ScanAggGraph(_RingGraph):
    def __init__(self, kernel: jit.Kernel, kd: NL.ColDesc, bucket_off, nb: int, grid: int,
                 GA: int, shmem: int, device, vec: int = 0):
        import torch
        from ..ops import kernels as K
        self.kernel = kernel
        self.kernels = (kernel,)
        self.kd = kd
        self.bucket_off = bucket_off
        self.nb, self.grid, self.GA, self.shmem = nb, grid, GA, shmem
        self.vec = vec   # rows per thread of a vectorized kernel (tiles over aligned ranges)
        self.tile = jit.BLOCK * (vec or jit.SCAN_ITEMS)
        # device intermediates are shared: replays on one stream execute in order
        self.d_params = torch.empty(PARAM_HEAD, dtype=torch.uint8, device=device)
        self.rstart = torch.empty(nb, dtype=torch.int64, device=device)
        self.rlen = torch.empty(nb, dtype=torch.int64, device=device)
        self.rbk = torch.empty(nb, dtype=torch.int32, device=device)
        self.tp = torch.empty(nb + 1, dtype=torch.int64, device=device)
        self.parts = jit._partials(grid, GA, device)
        self.out = K.agg_outputs(GA, device)
        self._init_ring(PARAM_HEAD)

    def _enqueue(self, slot: _Slot, stream: int, blocks) -> None:
        L = jit.runtime()
        K = NL.lib()
        NL.check(L.hs_memcpy_async(self.d_params.data_ptr(), slot.h_params.ptr,
                                   slot.h_params.nbytes, 1, stream), "param H2D")
        NL.check(K.hs_range_search_dev(C.byref(self.kd), NL.ptr(self.bucket_off), None, self.nb,
                                       self.d_params.data_ptr(), NL.ptr(self.rstart),
                                       NL.ptr(self.rlen), NL.ptr(self.rbk), stream),
                 "hs_range_search_dev")
        if self.vec:
            NL.check(K.hs_ranges_to_tiles_aligned(NL.ptr(self.rstart), NL.ptr(self.rlen), self.nb,
                                                  self.tile, self.vec, NL.ptr(self.tp), stream),
                     "hs_ranges_to_tiles_aligned")
        else:
            NL.check(K.hs_ranges_to_tiles(NL.ptr(self.rlen), self.nb, self.tile,
                                          NL.ptr(self.tp), stream), "hs_ranges_to_tiles")
        self.kernel.launch_packed(self.grid, blocks[0], stream, self.shmem)
        self._final_and_d2h(slot, stream, self.grid)

    def buffers(self) -> list:
        """Device intermediates a replay reads and writes."""
        return [self.d_params, self.rstart, self.rlen, self.rbk, self.tp, self.bucket_off,
                *self.parts, self.out[0].hs_buf]

    def values_template(self) -> dict:
        return {"rstart": self.rstart.data_ptr(), "rlen": self.rlen.data_ptr(),
                "tile_prefix": self.tp.data_ptr(), "R": self.nb,
                "psum": self.parts[0].data_ptr(), "pcnt": self.parts[1].data_ptr(),
                "pmin": self.parts[2].data_ptr(), "pmax": self.parts[3].data_ptr()}

    def launch(self, bounds: Tuple[int, int, int, int, int, int], args_block, stream=None,
               after=None) -> _Launch:
        """Queue one query on ``stream`` (default current), after ``after``'s queued work when
        given; ``result(handle)`` waits for it.  ``args_block``: the scan kernel's packed
        arguments (bytes or a ``_cbuf``)."""
        head = struct.pack("<6q", *bounds)

        def fill(hp):
            C.memmove(hp.ptr, head, 48)
        if not isinstance(args_block, C.Array):
            args_block = _cbuf(args_block)
        return self._launch_slot(fill, (args_block,), stream, after)

    def run(self, bounds: Tuple[int, int, int, int, int, int], args_block):
        """(sum, count, min, max) numpy arrays for one query (launch + wait)."""
        return self.result(self.launch(bounds, args_block))


def _nofill(hp) -> None:
    pass


class TwoPhaseGraph(_RingGraph):
    """The run-keyed two-phase merge-join aggregate (exec/jit_runs.py) captured: phase 1 (run
    tags), phase 2 (bits scan into the graph's partials), the deterministic final reduction and
    the result D2H - one replay per query instead of four launches and their host-side argument
    packing.  The tag bitmap and the run tables are the launcher's (fixed per lowering)."""

    def __init__(self, kt: jit.Kernel, ks: jit.Kernel, grid_t: int, grid_s: int, GA: int,
                 shmem: int, device):
        from ..ops import kernels as K
        self.kt, self.ks = kt, ks
        self.kernels = (kt, ks)
        self.grid_t, self.grid_s, self.GA, self.shmem = grid_t, grid_s, GA, shmem
        self.parts = jit._partials(grid_s, GA, device)
        self.out = K.agg_outputs(GA, device)
        self._init_ring(0)

    def _enqueue(self, slot: _Slot, stream: int, blocks) -> None:
        self.kt.launch_packed(self.grid_t, blocks[0], stream, 0)
        self.ks.launch_packed(self.grid_s, blocks[1], stream, self.shmem)
        self._final_and_d2h(slot, stream, self.grid_s)

    def buffers(self) -> list:
        return [*self.parts, self.out[0].hs_buf]

    def partial_ptrs(self) -> dict:
        return {"psum": self.parts[0].data_ptr(), "pcnt": self.parts[1].data_ptr(),
                "pmin": self.parts[2].data_ptr(), "pmax": self.parts[3].data_ptr()}

    def launch(self, block_t, block_s) -> _Launch:
        """``block_t`` / ``block_s``: ``_cbuf`` argument blocks of the two phases."""
        return self._launch_slot(_nofill, (block_t, block_s))


class GraphPending:
    """A replayed pipeline whose result block is still in flight."""
    __slots__ = ("graph", "handle")

    def __init__(self, graph, handle):
        self.graph, self.handle = graph, handle

    def result(self):
        return self.graph.result(self.handle)


class GraphCache:
    """Per-backend LRU of captured pipelines (graphs pin their buffers)."""

    def __init__(self, capacity: int = 64):
        self.capacity = capacity
        self._lru: "OrderedDict[tuple, ScanAggGraph]" = OrderedDict()
        self._lock = threading.Lock()

    def get(self, key: tuple, make) -> ScanAggGraph:
        with self._lock:
            g = self._lru.get(key)
            if g is not None:
                self._lru.move_to_end(key)
                return g
        g = make()
        with self._lock:
            self._lru[key] = g
            while len(self._lru) > self.capacity:
                _, old = self._lru.popitem(last=False)
                side = getattr(old, "side_stream", None)
                if side is not None:
                    # its last replays may still run on the side stream: let them finish before
                    # the executable graphs are destroyed
                    side.synchronize()
        return g

    def peek(self, key: tuple) -> Optional[ScanAggGraph]:
        """The cached pipeline of ``key`` (touched as most recent), or None."""
        with self._lock:
            g = self._lru.get(key)
            if g is not None:
                self._lru.move_to_end(key)
            return g

    def __len__(self):
        return len(self._lru)


def range_bounds(lo: Optional[int], lo_incl: bool, hi: Optional[int], hi_incl: bool):
    """The 6-int64 bound block read by ``hs_range_search_dev`` (images as signed int64 bits)."""
    def s64(v):
        v = int(v or 0) & 0xFFFFFFFFFFFFFFFF
        return v - (1 << 64) if v >= (1 << 63) else v
    return (1 if lo is not None else 0, s64(lo), 1 if lo_incl else 0,
            1 if hi is not None else 0, s64(hi), 1 if hi_incl else 0)
