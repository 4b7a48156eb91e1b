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
    from cdnaml.utils import Classroom
    from cdnaml.utils import datasets as D
    from cdnaml.utils.dbutils import to_local
    from cdnaml.utils.notebook import mount_dbfs_fuse, unmount_dbfs_fuse

    with session_device(request.param):
        root = tmp_path_factory.mktemp(f"parity_{request.param}")
        os.environ["CDNAML_DBFS_ROOT"] = str(root / "dbfs")
        os.environ["CDNAML_TRACKING_URI"] = str(root / "mlruns")
        spark = cdnaml.SparkSession.builder.config("cdnaml.warehouse.dir", str(root / "warehouse")).getOrCreate()
        assert spark.device.type == request.param
        installed = compat.install()
        # the notebooks' own path convention: f"{datasets_dir}/..." dbfs:/ URIs (Classroom-Setup.py:17-18) and
        # .replace("dbfs:/", "/dbfs/") for pandas (ML 05:69) -- every read and write goes through the resolver
        cr = Classroom(spark, lesson=f"parity {request.param}", install=False)
        D.install_datasets(to_local(cr.datasets_dir), spark, scale=0.03)
        mount_dbfs_fuse()
        try:
            yield spark, cr.datasets_dir, cr.working_dir
        finally:
            unmount_dbfs_fuse()
            compat.uninstall()
            spark.stop()
            del installed
