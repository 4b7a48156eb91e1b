"""Course-harness utilities: synthetic datasets, classroom helpers, dbutils/display."""
from .classroom import Classroom, get_username, path_exists, to_hash  # noqa: F401
from .datasets import install_datasets  # noqa: F401
from .dbutils import dbutils, display, displayHTML  # noqa: F401
from .notebook import mount_dbfs_fuse, notebook_namespace, run_notebook  # noqa: F401
