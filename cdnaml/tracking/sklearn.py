"""scikit-learn flavor (ML 05 - MLflow Model Registry.py:60-80; ML 12:27-42).

The pickle written here is produced by this framework's own ``save_model``;
``load_model`` only unpickles artifacts that this tracking store wrote.
"""
from __future__ import annotations

import os
import pickle

from .artifacts import resolve
from .models import Model, log_to_run, write_common

FLAVOR_NAME = "sklearn"


def save_model(sk_model, path, input_example=None, signature=None, run_id=None, artifact_path=None,
               serialization_format="pickle", **kw):
    os.makedirs(path, exist_ok=True)
    with open(os.path.join(path, "model.pkl"), "wb") as f:
        pickle.dump(sk_model, f)
    import sklearn
    m = Model(artifact_path, run_id, signature=signature)
    m.add_flavor(FLAVOR_NAME, pickled_model="model.pkl", sklearn_version=sklearn.__version__,
                 serialization_format=serialization_format, code=None)
    m.add_flavor("python_function", loader_module="cdnaml.tracking.sklearn", model_path="model.pkl",
                 env="conda.yaml", predict_fn="predict")
    write_common(path, m, input_example, ["scikit-learn", "numpy", "pandas"])


def log_model(sk_model, artifact_path, registered_model_name=None, input_example=None, signature=None, **kw):
    return log_to_run(lambda d, rid: save_model(sk_model, d, input_example, signature, rid, artifact_path),
                      artifact_path, registered_model_name)


def load_model(model_uri, dst_path=None):
    p = resolve(model_uri)
    with open(os.path.join(p, "model.pkl"), "rb") as f:
        return pickle.load(f)  # artifact written by save_model above


def _load_pyfunc(path):
    with open(path if path.endswith(".pkl") else os.path.join(path, "model.pkl"), "rb") as f:
        return pickle.load(f)


def autolog(**kw):
    pass
