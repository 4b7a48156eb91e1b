"""``mlflow.tracking`` namespace: ``MlflowClient`` and the tracking-URI helpers."""
from .client import MlflowClient  # noqa: F401
from .fluent import get_tracking_uri, is_tracking_uri_set, set_tracking_uri  # noqa: F401
from . import client  # noqa: F401
