from ..sql.functions import array_to_vector, vector_to_array  # noqa: F401
