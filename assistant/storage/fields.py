"""Portable 768-d embedding column.

The reference stores vectors with pgvector's ``VectorField`` + an HNSW index (storage/models.py:7-58).
Search no longer runs in the database (the exact in-HBM index of ``assistant.storage.index`` does it),
so the column only has to persist the vector: pgvector's type is used when pgvector is installed and
the database is PostgreSQL; otherwise the vector is stored as packed float32 bytes, which works on
SQLite/MySQL and in tests.  Python values are lists of floats (or numpy arrays) either way.
"""
from __future__ import annotations

import struct

import numpy as np
from django.db import models

try:  # pragma: no cover - optional dependency
    from pgvector.django import VectorField as _PgVectorField
except Exception:  # pgvector is optional
    _PgVectorField = None


class VectorField(models.Field):
    description = "fixed-size float vector"

    def __init__(self, *args, dimensions: int | None = None, **kwargs):
        self.dimensions = dimensions
        super().__init__(*args, **kwargs)

    def deconstruct(self):
        name, path, args, kwargs = super().deconstruct()
        if self.dimensions is not None:
            kwargs["dimensions"] = self.dimensions
        return name, "assistant.storage.fields.VectorField", args, kwargs

    def _pg(self, connection) -> bool:
        return _PgVectorField is not None and connection.vendor == "postgresql"

    def db_type(self, connection):
        if self._pg(connection):
            return f"vector({self.dimensions})" if self.dimensions else "vector"
        return connection.data_types.get("BinaryField", "blob")

    def get_db_prep_value(self, value, connection, prepared=False):
        if value is None:
            return None
        arr = np.asarray(value, dtype=np.float32).reshape(-1)
        if self.dimensions and arr.size != self.dimensions:
            raise ValueError(f"expected {self.dimensions} dimensions, got {arr.size}")
        if self._pg(connection):
            return "[" + ",".join(f"{x:.8g}" for x in arr.tolist()) + "]"
        return arr.tobytes()

    def from_db_value(self, value, expression, connection):
        return self.to_python(value)

    def to_python(self, value):
        if value is None or isinstance(value, list):
            return value
        if isinstance(value, np.ndarray):
            return value.astype(np.float32).tolist()
        if isinstance(value, (bytes, bytearray, memoryview)):
            b = bytes(value)
            return list(struct.unpack(f"<{len(b) // 4}f", b))
        if isinstance(value, str):
            return [float(x) for x in value.strip("[]").split(",") if x.strip()]
        return list(value)
