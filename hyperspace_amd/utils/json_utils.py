"""JSON helpers that reproduce the reference's Jackson output byte-for-byte in layout.

Reference: ``util/JsonUtils.scala:27-45`` — Jackson ``writerWithDefaultPrettyPrinter`` with
``Include.ALWAYS`` (nulls emitted).  Jackson's DefaultPrettyPrinter indents objects by two spaces
per nesting level, writes ``"key" : value``, keeps arrays inline (``[ a, b ]``, FixedSpaceIndenter,
which does *not* add a nesting level) and prints empty containers as ``{ }`` / ``[ ]``.
The canonical example this must match is ``IndexLogEntryTest.scala:83-185``.
"""
from __future__ import annotations

import json
from typing import Any


def _dump(value: Any, nesting: int, out: list) -> None:
    if isinstance(value, dict):
        if not value:
            out.append("{ }")
            return
        out.append("{")
        first = True
        for k, v in value.items():
            if not first:
                out.append(",")
            first = False
            out.append("\n")
            out.append("  " * (nesting + 1))
            out.append(json.dumps(str(k), ensure_ascii=False))
            out.append(" : ")
            _dump(v, nesting + 1, out)
        out.append("\n")
        out.append("  " * nesting)
        out.append("}")
    elif isinstance(value, (list, tuple)):
        if not value:
            out.append("[ ]")
            return
        out.append("[ ")
        for i, v in enumerate(value):
            if i:
                out.append(", ")
            _dump(v, nesting, out)
        out.append(" ]")
    elif value is None:
        out.append("null")
    elif isinstance(value, bool):
        out.append("true" if value else "false")
    elif isinstance(value, int):
        out.append(str(value))
    elif isinstance(value, float):
        out.append(repr(value))
    else:
        out.append(json.dumps(str(value), ensure_ascii=False))


def to_json(value: Any) -> str:
    """Serialize a JSON-compatible python value with Jackson's default pretty printer layout."""
    if hasattr(value, "to_json_obj"):
        value = value.to_json_obj()
    out: list = []
    _dump(value, 0, out)
    return "".join(out)


def json_to_map(text: str) -> dict:
    return json.loads(text)


def from_json(text: str) -> Any:
    return json.loads(text)


def compact(value: Any) -> str:
    """Compact JSON as produced by Spark's ``DataType.json`` (no whitespace)."""
    return json.dumps(value, separators=(",", ":"), ensure_ascii=False)
