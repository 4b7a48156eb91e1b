from ..models.linalg import DenseMatrix, DenseVector, Matrices, SparseVector, Vector, Vectors  # noqa: F401
from ..sql.types import VectorUDT  # noqa: F401
