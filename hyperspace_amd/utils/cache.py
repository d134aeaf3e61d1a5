"""``CacheWithTransform`` (reference ``util/CacheWithTransform.scala:31-45``).

Memoizes ``transform(init())`` and recomputes only when ``init()`` returns a new value — used for
conf-driven lists (source builders, supported formats) that must react to conf changes.
"""
from __future__ import annotations


class CacheWithTransform:
    _UNSET = object()

    def __init__(self, init_fn, transform_fn):
        self._init = init_fn
        self._transform = transform_fn
        self._key = self._UNSET
        self._value = None

    def load(self):
        key = self._init()
        if self._key is self._UNSET or key != self._key:
            self._value = self._transform(key)
            self._key = key
        return self._value
