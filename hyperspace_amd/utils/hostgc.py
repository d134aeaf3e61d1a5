"""Keeping CPython's cyclic garbage collector off the serving loop's host path.

A serving loop allocates a few hundred short-lived objects per query (the DataFrame, its
expression tree, the future) and frees them by reference counting, yet every ~70k net
allocations the collector promotes and, every tenth gen-1 pass, runs a full collection over
*every* tracked object of the process - the engine's plans, lowerings, captured graphs and the
Arrow / torch objects around them.  Measured with ``scripts/diag/host_path.py --phases``: one
full pass costs ~100+ ms of host time on this container's CPU, landing inside whichever query
triggers it.

``settle()`` runs when the engine has just built long-lived state (a query shape's prepared
program, exec/gpu.py ``_register_program``): a young-generation collection, then ``gc.freeze()``,
which moves everything alive into the permanent generation that later collections skip.
Objects frozen stay until they are freed by reference counting (cyclic garbage among them is not
reclaimed), so it runs once per new shape, not per query.  Conf:
``spark.hyperspace.mi.host.gcFreeze.enabled`` (default true).
"""
from __future__ import annotations

import gc

STATS = {"settles": 0}


def settle() -> None:
    gc.collect(1)
    gc.freeze()
    STATS["settles"] += 1
