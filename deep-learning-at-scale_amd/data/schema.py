"""Schema strings of the submission contract (cnn.py:41-44, 53-62, 72, 93).

The submission passes two comma-separated strings of equal length: column names and
column types. The reference maps each type with a tuple-index trick (cnn.py:55-59):
``"int"`` -> IntegerType, ``"float"`` -> FloatType and ANYTHING else -> StringType
(so ``"double"`` becomes a string column). All fields are nullable. That exact mapping
is kept here, including the catch-all, because web-side job submitters depend on it.
"""
from __future__ import annotations

import dataclasses

INT, FLOAT, STRING = "int", "float", "string"


@dataclasses.dataclass(frozen=True)
class Field:
    name: str
    kind: str  # INT | FLOAT | STRING
    nullable: bool = True

    @property
    def is_numeric(self) -> bool:
        return self.kind in (INT, FLOAT)

    def spark_repr(self) -> str:
        t = {INT: "IntegerType()", FLOAT: "FloatType()", STRING: "StringType()"}[self.kind]
        return f"StructField('{self.name}', {t}, {self.nullable})"


@dataclasses.dataclass(frozen=True)
class Schema:
    fields: tuple

    @property
    def names(self):
        return [f.name for f in self.fields]

    def __getitem__(self, name: str) -> Field:
        for f in self.fields:
            if f.name == name:
                return f
        raise KeyError(name)

    def categorical(self, exclude=()):
        """cnn.py:72 — type neither int nor float (target excluded: defect A.1#4 fixed)."""
        return [f.name for f in self.fields if not f.is_numeric and f.name not in exclude]

    def continuous(self, exclude=()):
        """cnn.py:93 — int or float columns, in schema order, minus ``exclude``."""
        return [f.name for f in self.fields if f.is_numeric and f.name not in exclude]

    def __str__(self) -> str:  # what cnn.py:62 printed
        return "StructType([" + ", ".join(f.spark_repr() for f in self.fields) + "])"


def map_type(v: str) -> str:
    """cnn.py:55-59 semantics: 'int' -> int, 'float' -> float, else -> string."""
    v = v.strip()
    if v == "int":
        return INT
    if v == "float":
        return FLOAT
    return STRING


def parse_schema(column_names: str, column_types: str) -> Schema:
    names = [n.strip() for n in column_names.split(",")]
    types = column_types.split(",")
    if len(names) != len(types):
        # the reference zips silently (truncating); a mismatch is always a caller bug
        raise ValueError(f"{len(names)} column names but {len(types)} column types")
    if len(set(names)) != len(names):
        raise ValueError("duplicate column names")
    return Schema(tuple(Field(n, map_type(t)) for n, t in zip(names, types)))
