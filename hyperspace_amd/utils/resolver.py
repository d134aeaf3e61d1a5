"""Column-name resolution honouring ``spark.sql.caseSensitive`` (reference
``util/ResolverUtils.scala:25-74``)."""
from __future__ import annotations

from typing import Iterable, Optional, Sequence


def _eq(a: str, b: str, case_sensitive: bool) -> bool:
    return a == b if case_sensitive else a.lower() == b.lower()


def resolve_one(name: str, available: Iterable[str], case_sensitive: bool = False) -> Optional[str]:
    for a in available:
        if _eq(name, a, case_sensitive):
            return a
    return None


def resolve(names: Sequence[str], available: Sequence[str],
            case_sensitive: bool = False) -> Optional[list]:
    """Resolve all names; ``None`` if any fails (``ResolverUtils.scala:68-73``)."""
    out = []
    avail = list(available)
    for n in names:
        r = resolve_one(n, avail, case_sensitive)
        if r is None:
            return None
        out.append(r)
    return out
