"""Row -> Table transformation for tabular data (reference S/dataset/datamining/RowTransformer.scala:44-330).

A row is a mapping of field name -> value (a pandas row, a dict, or a (values, field_names) pair standing in for
Spark SQL's Row + schema). Each ``RowTransform`` produces one tensor under its schema key:
``ColsToNumeric`` concatenates numeric fields into one float tensor, ``ColToTensor`` turns one field into a tensor
(atomic fields: strings stay Python values wrapped in a list tensor-like). The result is a Table keyed by schema
key, the shape the reference's feature-engineering ops consume.
"""
import torch

from ..utils.table import Table
from .core import Transformer


def _as_dict(row, fieldNames=None):
    if isinstance(row, dict):
        return row
    if hasattr(row, "to_dict"):
        return row.to_dict()
    if isinstance(row, tuple) and len(row) == 2 and isinstance(row[1], (list, tuple)):
        vals, names = row
        return dict(zip(names, vals))
    if fieldNames is not None:
        return dict(zip(fieldNames, row))
    raise TypeError("row must be a dict, a pandas row, or (values, field_names)")


class RowTransform:
    def __init__(self, schemaKey, fieldNames=None):
        self.schemaKey = schemaKey
        self.fieldNames = list(fieldNames) if fieldNames is not None else None

    def transform(self, values):
        raise NotImplementedError


class ColsToNumeric(RowTransform):
    """Selected (or all numeric) fields -> one 1-D float tensor."""

    def __init__(self, schemaKey, fieldNames=None, dtype=torch.float32):
        super().__init__(schemaKey, fieldNames)
        self.dtype = dtype

    def transform(self, values):
        vals = [values[k] for k in self.fieldNames] if self.fieldNames else \
            [v for v in values.values() if isinstance(v, (int, float, bool))]
        return torch.tensor([float(v) for v in vals], dtype=self.dtype)


class ColToTensor(RowTransform):
    """One field -> a tensor (numbers / arrays) or the raw value (strings: the reference's Tensor[String])."""

    def __init__(self, schemaKey, fieldName):
        super().__init__(schemaKey, [fieldName])

    def transform(self, values):
        v = values[self.fieldNames[0]]
        if isinstance(v, str):
            return [v]
        return torch.as_tensor(v).reshape(-1) if not isinstance(v, torch.Tensor) else v.reshape(-1)


class RowTransformer(Transformer):
    def __init__(self, schema, rowSize=None, fieldNames=None):
        self.schema = list(schema)
        self.rowSize = rowSize
        self.fieldNames = fieldNames
        keys = [s.schemaKey for s in self.schema]
        if len(set(keys)) != len(keys):
            raise ValueError("schema keys must be unique")

    def apply(self, it):
        for row in it:
            d = _as_dict(row, self.fieldNames)
            if self.rowSize is not None and len(d) != self.rowSize:
                raise ValueError(f"row size {len(d)} != {self.rowSize}")
            t = Table()
            for s in self.schema:
                t[s.schemaKey] = s.transform(d)
            yield t

    # factories (RowTransformer.scala:98-206)
    @staticmethod
    def atomic(fieldNames):
        return RowTransformer([ColToTensor(n, n) for n in fieldNames])

    @staticmethod
    def numeric(numericFields=None, schemaKey="all"):
        if numericFields is None:
            return RowTransformer([ColsToNumeric(schemaKey)])
        return RowTransformer([ColsToNumeric(k, v) for k, v in numericFields.items()])

    @staticmethod
    def atomicWithNumeric(atomicFields, numericFields):
        return RowTransformer([ColToTensor(n, n) for n in atomicFields] +
                              [ColsToNumeric(k, v) for k, v in numericFields.items()])


__all__ = ["RowTransformer", "RowTransform", "ColsToNumeric", "ColToTensor"]
