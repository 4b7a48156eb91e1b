from ..models.recommendation import ALS, ALSModel  # noqa: F401
