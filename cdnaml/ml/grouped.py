from ..models.grouped import GroupedEstimator, GroupedModel  # noqa: F401
