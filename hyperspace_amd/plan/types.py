"""Schema / type system: pyarrow schemas inside the engine, Spark ``StructType.json`` on disk.

``schemaString`` and ``dataSchemaJson`` in the index log (``IndexLogEntry.scala:347-360,409-414``)
are Spark DataType JSON; this module converts both ways so logs stay interchangeable with
reference-built indexes.
"""
from __future__ import annotations

import re

import pyarrow as pa

from ..utils import json_utils

_SIMPLE_TO_SPARK = [
    (pa.types.is_boolean, "boolean"),
    (lambda t: pa.types.is_int8(t), "byte"),
    (lambda t: pa.types.is_int16(t), "short"),
    (lambda t: pa.types.is_int32(t), "integer"),
    (lambda t: pa.types.is_int64(t), "long"),
    (lambda t: pa.types.is_uint8(t), "short"),
    (lambda t: pa.types.is_uint16(t), "integer"),
    (lambda t: pa.types.is_uint32(t), "long"),
    (lambda t: pa.types.is_uint64(t), "long"),
    (pa.types.is_float32, "float"),
    (pa.types.is_float64, "double"),
    (pa.types.is_float16, "float"),
    (lambda t: pa.types.is_string(t) or pa.types.is_large_string(t), "string"),
    (lambda t: pa.types.is_binary(t) or pa.types.is_large_binary(t), "binary"),
    (pa.types.is_date32, "date"),
    (pa.types.is_date64, "date"),
    (pa.types.is_timestamp, "timestamp"),
    (pa.types.is_null, "null"),
]

_SPARK_TO_ARROW = {
    "boolean": pa.bool_(), "byte": pa.int8(), "short": pa.int16(), "integer": pa.int32(),
    "long": pa.int64(), "float": pa.float32(), "double": pa.float64(), "string": pa.string(),
    "binary": pa.binary(), "date": pa.date32(), "timestamp": pa.timestamp("us"),
    "null": pa.null(),
}


def spark_type_json(t: pa.DataType):
    if pa.types.is_dictionary(t):
        return spark_type_json(t.value_type)
    if pa.types.is_decimal(t):
        return f"decimal({t.precision},{t.scale})"
    for pred, name in _SIMPLE_TO_SPARK:
        if pred(t):
            return name
    if pa.types.is_list(t) or pa.types.is_large_list(t):
        return {"type": "array", "elementType": spark_type_json(t.value_type), "containsNull": True}
    if pa.types.is_struct(t):
        return {"type": "struct", "fields": [_field_json(t.field(i)) for i in range(t.num_fields)]}
    if pa.types.is_map(t):
        return {"type": "map", "keyType": spark_type_json(t.key_type),
                "valueType": spark_type_json(t.item_type), "valueContainsNull": True}
    raise TypeError(f"unsupported arrow type {t}")


def _field_json(f: pa.Field):
    return {"name": f.name, "type": spark_type_json(f.type), "nullable": bool(f.nullable),
            "metadata": {}}


def schema_to_json(schema: pa.Schema) -> str:
    return json_utils.compact({"type": "struct", "fields": [_field_json(f) for f in schema]})


def spark_type_to_arrow(t) -> pa.DataType:
    if isinstance(t, str):
        m = re.fullmatch(r"decimal\((\d+),\s*(\d+)\)", t)
        if m:
            return pa.decimal128(int(m.group(1)), int(m.group(2)))
        if t == "decimal":
            return pa.decimal128(10, 0)
        return _SPARK_TO_ARROW[t]
    kind = t["type"]
    if kind == "array":
        return pa.list_(spark_type_to_arrow(t["elementType"]))
    if kind == "struct":
        return pa.struct([pa.field(f["name"], spark_type_to_arrow(f["type"]), f.get("nullable", True))
                          for f in t["fields"]])
    if kind == "map":
        return pa.map_(spark_type_to_arrow(t["keyType"]), spark_type_to_arrow(t["valueType"]))
    raise TypeError(f"unsupported spark type {t}")


def schema_from_json(text: str) -> pa.Schema:
    o = json_utils.from_json(text)
    return pa.schema([pa.field(f["name"], spark_type_to_arrow(f["type"]), f.get("nullable", True))
                      for f in o["fields"]])


def simple_string(t: pa.DataType) -> str:
    """Spark ``DataType.simpleString`` (used in explain's ReadSchema)."""
    j = spark_type_json(t)
    if isinstance(j, str):
        return {"integer": "int", "long": "bigint", "short": "smallint", "byte": "tinyint"}.get(j, j)
    if j["type"] == "array":
        return f"array<{simple_string(t.value_type)}>"
    if j["type"] == "struct":
        return "struct<" + ",".join(f"{f.name}:{simple_string(f.type)}" for f in t) + ">"
    return str(j["type"])


def struct_string(schema: pa.Schema) -> str:
    return "struct<" + ",".join(f"{f.name}:{simple_string(f.type)}" for f in schema) + ">"


def is_numeric(t: pa.DataType) -> bool:
    return pa.types.is_integer(t) or pa.types.is_floating(t) or pa.types.is_decimal(t)


def common_numeric(a: pa.DataType, b: pa.DataType) -> pa.DataType:
    if pa.types.is_floating(a) or pa.types.is_floating(b) or pa.types.is_decimal(a) or \
            pa.types.is_decimal(b):
        return pa.float64()
    if pa.types.is_integer(a) and pa.types.is_integer(b):
        return pa.int64() if max(a.bit_width, b.bit_width) > 32 else pa.int32()
    return pa.float64()
