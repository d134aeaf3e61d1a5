"""Staleness signatures (reference ``LogicalPlanSignatureProvider.scala:27-63``,
``FileBasedSignatureProvider.scala:31-62``, ``PlanSignatureProvider.scala:28-44``,
``IndexSignatureProvider.scala:33-51``).

Provider names stored in the log are the reference's JVM class names, so signatures written by
either engine validate in both.
"""
from __future__ import annotations

from typing import Optional

from ..utils.hashing import md5_hex

INDEX_SIGNATURE_PROVIDER = "com.microsoft.hyperspace.index.IndexSignatureProvider"
FILE_BASED_SIGNATURE_PROVIDER = "com.microsoft.hyperspace.index.FileBasedSignatureProvider"
PLAN_SIGNATURE_PROVIDER = "com.microsoft.hyperspace.index.PlanSignatureProvider"


class LogicalPlanSignatureProvider:
    name = ""

    def signature(self, plan, session=None) -> Optional[str]:
        raise NotImplementedError


def _session(session):
    if session is not None:
        return session
    from ..session import Session
    return Session.active()


class FileBasedSignatureProvider(LogicalPlanSignatureProvider):
    name = FILE_BASED_SIGNATURE_PROVIDER

    def signature(self, plan, session=None):
        from ..hyperspace import get_context
        from ..plan.logical import LogicalRelation
        mgr = get_context(_session(session)).source_provider_manager
        fp = []
        plan.foreach_up(lambda p: fp.append(mgr.signature(p)) if isinstance(p, LogicalRelation)
                        else None)
        s = "".join(fp)
        return md5_hex(s) if s else None


class PlanSignatureProvider(LogicalPlanSignatureProvider):
    name = PLAN_SIGNATURE_PROVIDER

    def signature(self, plan, session=None):
        acc = [""]
        plan.foreach_up(lambda p: acc.__setitem__(0, md5_hex(acc[0] + p.node_name)))
        return acc[0] or None


class IndexSignatureProvider(LogicalPlanSignatureProvider):
    name = INDEX_SIGNATURE_PROVIDER

    def signature(self, plan, session=None):
        f = FileBasedSignatureProvider().signature(plan, session)
        if f is None:
            return None
        p = PlanSignatureProvider().signature(plan, session)
        return None if p is None else md5_hex(f + p)


_REGISTRY = {
    INDEX_SIGNATURE_PROVIDER: IndexSignatureProvider,
    FILE_BASED_SIGNATURE_PROVIDER: FileBasedSignatureProvider,
    PLAN_SIGNATURE_PROVIDER: PlanSignatureProvider,
}


def create(name: Optional[str] = None) -> LogicalPlanSignatureProvider:
    if name is None:
        return IndexSignatureProvider()
    cls = _REGISTRY.get(name)
    if cls is None:
        try:
            import importlib
            mod, _, c = name.rpartition(".")
            cls = getattr(importlib.import_module(mod), c)
        except Exception as e:  # noqa: BLE001
            raise ValueError(f"Signature provider with name {name} is not supported.") from e
    inst = cls()
    if not hasattr(inst, "signature"):
        raise ValueError(f"Signature provider with name {name} is not supported.")
    return inst


def register(name: str, cls) -> None:
    _REGISTRY[name] = cls
