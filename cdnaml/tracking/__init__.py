"""MLflow-compatible tracking, model registry and model flavors (file store)."""
