"""Notebook-parity suite: one flow per reference notebook, written with the
reference's own imports (pyspark / mlflow / hyperopt / delta / koalas / databricks.*) through
``cdnaml.compat.install()``, on the synthetic course datasets (``cdnaml.utils.datasets``), asserting
the invariants each notebook states or implies."""
import os

import pytest

from tests.conftest import DEVICES, session_device


@pytest.fixture(scope="module", params=DEVICES)
def nb(request, tmp_path_factory):
    """(spark, datasets_root, workdir) with the compat aliases installed for the module; every flow runs on the
    host (CPU suite) and on the GPU (the cuda variant is marked gpu)."""
    import cdnaml
    import cdnaml.compat as compat
    from cdnaml.utils import datasets as D

    with session_device(request.param):
        root = tmp_path_factory.mktemp(f"parity_{request.param}")
        os.environ["CDNAML_DBFS_ROOT"] = str(root / "dbfs")
        os.environ["CDNAML_TRACKING_URI"] = str(root / "mlruns")
        spark = cdnaml.SparkSession.builder.config("cdnaml.warehouse.dir", str(root / "warehouse")).getOrCreate()
        assert spark.device.type == request.param
        installed = compat.install()
        ds = D.install_datasets(str(root / "datasets"), spark, scale=0.03)
        try:
            yield spark, ds, str(root / "work")
        finally:
            compat.uninstall()
            spark.stop()
            del installed
