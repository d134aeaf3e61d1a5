"""Keeping CPython's cyclic garbage collector off the serving loop's host path.

A serving loop allocates a few hundred short-lived objects per query (the DataFrame, its
expression tree, the future) and frees them by reference counting, yet every ~70k net
allocations the collector promotes and, every tenth gen-1 pass, runs a full collection over
*every* tracked object of the process - the engine's plans, lowerings, captured graphs and the
Arrow / torch objects around them.  Measured with ``scripts/diag/host_path.py --phases``: one
full pass costs ~100+ ms of host time on this container's CPU, landing inside whichever query
triggers it.

``settle()`` moves everything alive into the permanent generation (``gc.freeze()``) that
later collections skip:

* ``settle(full=True)`` when Hyperspace is enabled on a session (``Session.enableHyperspace``,
  the start of a serving phase): the previous freeze is undone and one full collection runs
  first, so cyclic garbage frozen earlier (a dropped session, a replaced table) is reclaimed
  there - frozen objects are otherwise only freed by reference counting;
* ``settle()`` when the engine has just built a query shape's long-lived state (its prepared
  program, exec/gpu.py ``_register_program``): a young-generation collection, then the freeze.

Conf: ``spark.hyperspace.mi.host.gcFreeze.enabled`` (default true).
"""
from __future__ import annotations

import gc

STATS = {"settles": 0, "full": 0}


def settle(full: bool = False) -> None:
    if full:
        gc.unfreeze()
        gc.collect()
        STATS["full"] += 1
    else:
        gc.collect(1)
    gc.freeze()
    STATS["settles"] += 1
