"""pyspark.ml.linalg surface: dense / sparse vectors and matrices (Spark's CSC layout)."""
import numpy as np

from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.linalg import (DenseMatrix, DenseVector, Matrices,
                                                                                SparseMatrix, Vectors)


def test_sparse_matrix_csc_layout():
    # Spark doc example: Matrices.sparse(2, 2, [0, 2, 3], [0, 1, 1], [2, 3, 4]) = [[2, 0], [3, 4]]
    m = Matrices.sparse(2, 2, [0, 2, 3], [0, 1, 1], [2, 3, 4])
    np.testing.assert_array_equal(m.toArray(), [[2, 0], [3, 4]])
    assert m[1, 0] == 3.0 and m == m.toDense()
    d = DenseMatrix(2, 3, [1, 0, 0, 5, 7, 0])
    s = d.toSparse()
    assert isinstance(s, SparseMatrix) and s.colPtrs.tolist() == [0, 1, 2, 3]
    np.testing.assert_array_equal(s.toArray(), d.toArray())
    t = SparseMatrix(2, 2, [0, 1, 2], [1, 0], [9, 8], isTransposed=True)
    np.testing.assert_array_equal(t.toArray(), [[0, 9], [8, 0]])


def test_vectors():
    v = Vectors.sparse(4, [1, 3], [3.0, 4.0])
    assert v.dot([1, 1, 1, 1]) == 7.0 and v.norm(2) == 5.0
    assert v.toDense() == DenseVector([0, 3, 0, 4]) and DenseVector([0, 3, 0, 4]).toSparse() == v
    assert Vectors.squared_distance([1, 2], [3, 4]) == 8.0
    np.testing.assert_array_equal((-DenseVector([1, 2])).toArray(), [-1, -2])
    np.testing.assert_array_equal((2 * DenseVector([1, 2])).toArray(), [2, 4])
