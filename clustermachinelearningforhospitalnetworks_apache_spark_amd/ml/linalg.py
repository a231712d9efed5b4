"""pyspark.ml.linalg-compatible vectors and matrices (host objects).

Vector *columns* never hold these objects: a ``features`` column is one dense
[n, d] tensor resident on the rank's device.  These classes exist for the
user-facing API: ``Row.features``, ``model.coefficients``,
``model.clusterCenters()``, ``featureImportances`` (ref.py:230-235) and the
VectorUDT/MatrixUDT structs of the Parquet model format.
"""
from __future__ import annotations

from typing import Dict, Iterable, List, Optional, Sequence, Tuple, Union

import numpy as np


class Vector:
    def toArray(self) -> np.ndarray:
        raise NotImplementedError

    @property
    def size(self) -> int:
        raise NotImplementedError

    def __len__(self):
        return self.size

    def __iter__(self):
        return iter(self.toArray())

    def __array__(self, dtype=None, copy=None):
        a = self.toArray()
        return a.astype(dtype) if dtype is not None else a

    def dot(self, other) -> float:
        return float(np.dot(self.toArray(), np.asarray(other, dtype=np.float64)))

    def norm(self, p) -> float:
        return float(np.linalg.norm(self.toArray(), p))

    def squared_distance(self, other) -> float:
        d = self.toArray() - np.asarray(other, dtype=np.float64)
        return float(d @ d)


class DenseVector(Vector):
    def __init__(self, ar: Union[Sequence[float], np.ndarray]):
        self.array = np.asarray(ar, dtype=np.float64).reshape(-1)

    def toArray(self) -> np.ndarray:
        return self.array

    @property
    def values(self) -> np.ndarray:
        return self.array

    @property
    def size(self) -> int:
        return int(self.array.shape[0])

    def numNonzeros(self) -> int:
        return int(np.count_nonzero(self.array))

    def __getitem__(self, i):
        return self.array[i]

    def __eq__(self, other):
        if isinstance(other, Vector):
            return np.array_equal(self.toArray(), other.toArray())
        return False

    def __hash__(self):
        return hash(self.array.tobytes())

    def __repr__(self):
        return f"DenseVector([{', '.join(repr(float(v)) for v in self.array)}])"

    def __str__(self):
        return "[" + ",".join(repr(float(v)) for v in self.array) + "]"

    def __add__(self, o):
        return DenseVector(self.array + np.asarray(o, dtype=np.float64))

    def __sub__(self, o):
        return DenseVector(self.array - np.asarray(o, dtype=np.float64))

    def __mul__(self, o):
        return DenseVector(self.array * np.asarray(o, dtype=np.float64))

    def __truediv__(self, o):
        return DenseVector(self.array / np.asarray(o, dtype=np.float64))

    def __neg__(self):
        return DenseVector(-self.array)

    __radd__ = __add__
    __rmul__ = __mul__

    def toSparse(self) -> "SparseVector":
        nz = np.nonzero(self.array)[0]
        return SparseVector(self.size, nz.tolist(), self.array[nz].tolist())


class SparseVector(Vector):
    def __init__(self, size: int, *args):
        self._size = int(size)
        if len(args) == 1:
            pairs = args[0]
            if isinstance(pairs, dict):
                pairs = sorted(pairs.items())
            idx = [int(i) for i, _ in pairs]
            val = [float(v) for _, v in pairs]
        else:
            idx, val = args
        order = np.argsort(np.asarray(idx, dtype=np.int64), kind="stable")
        self.indices = np.asarray(idx, dtype=np.int32)[order]
        self.values = np.asarray(val, dtype=np.float64)[order]

    @property
    def size(self) -> int:
        return self._size

    def toArray(self) -> np.ndarray:
        a = np.zeros(self._size)
        a[self.indices] = self.values
        return a

    def numNonzeros(self) -> int:
        return int(np.count_nonzero(self.values))

    def toDense(self) -> DenseVector:
        return DenseVector(self.toArray())

    def dot(self, other) -> float:
        o = as_array(other)
        return float(np.dot(self.values, o[self.indices]))

    def __getitem__(self, i):
        return self.toArray()[i]

    def __eq__(self, other):
        if isinstance(other, Vector):
            return np.array_equal(self.toArray(), other.toArray())
        return False

    def __hash__(self):
        return hash(self.toArray().tobytes())

    def __repr__(self):
        return f"SparseVector({self._size}, {{{', '.join(f'{i}: {v!r}' for i, v in zip(self.indices, self.values))}}})"

    def __str__(self):
        return f"({self._size},[{','.join(map(str, self.indices))}],[{','.join(repr(float(v)) for v in self.values)}])"


class Vectors:
    @staticmethod
    def dense(*elements) -> DenseVector:
        if len(elements) == 1 and not isinstance(elements[0], (int, float, np.floating, np.integer)):
            return DenseVector(elements[0])
        return DenseVector(list(elements))

    @staticmethod
    def sparse(size: int, *args) -> SparseVector:
        return SparseVector(size, *args)

    @staticmethod
    def zeros(size: int) -> DenseVector:
        return DenseVector(np.zeros(size))

    @staticmethod
    def norm(vector, p) -> float:
        return float(np.linalg.norm(np.asarray(vector, dtype=np.float64), p))

    @staticmethod
    def squared_distance(v1, v2) -> float:
        d = np.asarray(v1, dtype=np.float64) - np.asarray(v2, dtype=np.float64)
        return float(d @ d)


class Matrix:
    def __init__(self, numRows: int, numCols: int, isTransposed: bool = False):
        self.numRows = numRows
        self.numCols = numCols
        self.isTransposed = isTransposed


class DenseMatrix(Matrix):
    """Column-major dense matrix (Spark's layout; isTransposed => row-major values)."""

    def __init__(self, numRows: int, numCols: int, values, isTransposed: bool = False):
        super().__init__(numRows, numCols, isTransposed)
        self.values = np.asarray(values, dtype=np.float64).reshape(-1)

    def toArray(self) -> np.ndarray:
        if self.isTransposed:
            return self.values.reshape(self.numRows, self.numCols)
        return self.values.reshape(self.numCols, self.numRows).T

    def __eq__(self, other):
        return isinstance(other, Matrix) and np.array_equal(self.toArray(), other.toArray())

    def __getitem__(self, ij):
        i, j = ij
        return float(self.toArray()[i, j])

    def toSparse(self) -> "SparseMatrix":
        return SparseMatrix.from_dense(self.toArray())

    def __repr__(self):
        return f"DenseMatrix({self.numRows}, {self.numCols}, {self.values.tolist()}, {self.isTransposed})"


class SparseMatrix(Matrix):
    """Compressed sparse column matrix (Spark's layout; isTransposed => compressed rows)."""

    def __init__(self, numRows: int, numCols: int, colPtrs, rowIndices, values, isTransposed: bool = False):
        super().__init__(numRows, numCols, isTransposed)
        self.colPtrs = np.asarray(colPtrs, dtype=np.int32)
        self.rowIndices = np.asarray(rowIndices, dtype=np.int32)
        self.values = np.asarray(values, dtype=np.float64)
        major = numRows if isTransposed else numCols
        if self.colPtrs.shape[0] != major + 1:
            raise ValueError(f"colPtrs must have {major + 1} entries")
        if self.rowIndices.shape[0] != self.values.shape[0]:
            raise ValueError("rowIndices and values differ in length")

    @staticmethod
    def from_dense(a: np.ndarray) -> "SparseMatrix":
        a = np.asarray(a, dtype=np.float64)
        ptrs, rows, vals = [0], [], []
        for j in range(a.shape[1]):
            nz = np.nonzero(a[:, j])[0]
            rows.extend(nz.tolist())
            vals.extend(a[nz, j].tolist())
            ptrs.append(len(rows))
        return SparseMatrix(a.shape[0], a.shape[1], ptrs, rows, vals)

    def toArray(self) -> np.ndarray:
        major, minor = (self.numRows, self.numCols) if self.isTransposed else (self.numCols, self.numRows)
        out = np.zeros((minor, major))
        for j in range(major):
            a, b = self.colPtrs[j], self.colPtrs[j + 1]
            out[self.rowIndices[a:b], j] = self.values[a:b]
        return out.T if self.isTransposed else out

    def toDense(self) -> DenseMatrix:
        return Matrices.from_numpy(self.toArray())

    def __getitem__(self, ij):
        i, j = ij
        return float(self.toArray()[i, j])

    def __eq__(self, other):
        return isinstance(other, Matrix) and np.array_equal(self.toArray(), other.toArray())

    def __repr__(self):
        return (f"SparseMatrix({self.numRows}, {self.numCols}, {self.colPtrs.tolist()}, {self.rowIndices.tolist()}, "
                f"{self.values.tolist()}, {self.isTransposed})")


class Matrices:
    @staticmethod
    def dense(numRows: int, numCols: int, values) -> DenseMatrix:
        return DenseMatrix(numRows, numCols, values)

    @staticmethod
    def sparse(numRows: int, numCols: int, colPtrs, rowIndices, values) -> SparseMatrix:
        return SparseMatrix(numRows, numCols, colPtrs, rowIndices, values)

    @staticmethod
    def from_numpy(a: np.ndarray) -> DenseMatrix:
        a = np.asarray(a, dtype=np.float64)
        return DenseMatrix(a.shape[0], a.shape[1], a.T.reshape(-1), False)


def as_array(v) -> np.ndarray:
    if isinstance(v, Vector):
        return v.toArray()
    return np.asarray(v, dtype=np.float64)
