"""Databricks notebook runtime (§4 item 3): run the
reference's notebook-source ``.py`` files UNCHANGED on this engine.

A Databricks notebook starts with ``spark``, ``sc``, ``sql``, ``table``,
``display``, ``displayHTML`` and ``dbutils`` predefined, and every course
notebook then does ``%run ./Includes/Classroom-Setup``
(``Includes/Classroom-Setup.py:2-110``), which defines ``username``,
``userhome``, ``datasets_dir``, ``working_dir``, the answer validators of
``Includes/Class-Utility-Methods.py:15-363`` and ``install_datasets``.

* ``notebook_namespace()`` returns exactly that global namespace, backed by
  :class:`~cdnaml.utils.classroom.Classroom` (synthetic datasets, H2).
* ``mount_dbfs_fuse()`` emulates the ``/dbfs`` FUSE mount for pandas, which
  the notebooks use as ``pd.read_csv(path.replace("dbfs:/", "/dbfs/"))``
  (``ML 05:69``, ``ML 12:34``, ``ML 14:96``, ``Labs/ML 08L:34``): when the DBFS
  root is not literally ``/dbfs`` the pandas readers/writers get a path
  translation through the one resolver ``dbutils.to_local``.  It is opt-in
  (only notebook runs install it) and ``unmount_dbfs_fuse()`` restores pandas.
* ``split_cells()`` / ``run_notebook()`` execute the source cell by cell:
  Python cells verbatim, ``%sql`` cells through ``spark.sql`` (and
  materialised), ``%run ./Includes/...`` through the namespace, ``%md`` /
  ``%pip`` skipped.

CLI (one process, many notebooks -- the GPU suite uses this so a single
process owns the card)::

    python -m cdnaml.utils.notebook --scale 0.05 --json out.json "ML 02 - Linear Regression I.py" ...
"""
from __future__ import annotations

import io
import json
import os
import re
import sys
import time
import traceback
from contextlib import redirect_stdout
from dataclasses import asdict, dataclass, field
from typing import Any, Callable, Dict, List, Optional, Tuple

from .dbutils import dbutils, to_local

# ---------------------------------------------------------------- /dbfs FUSE

_PANDAS_READERS = ("read_csv", "read_parquet", "read_json", "read_table")
_PANDAS_WRITERS = ("to_csv", "to_parquet", "to_json")
_fuse_saved: Dict[Tuple[str, str], Any] = {}


def _fuse_path(p):
    if isinstance(p, str) and (p.startswith("/dbfs/") or p.startswith("dbfs:") or p.startswith("file:/dbfs")):
        return to_local(p)
    return p


def mount_dbfs_fuse() -> bool:
    """Make ``/dbfs/x`` readable/writable by pandas as ``<dbfs_root>/x``.

    Returns False (nothing installed) when the DBFS root IS ``/dbfs``."""
    from .dbutils import dbfs_root
    if dbfs_root() == "/dbfs" or _fuse_saved:
        return False
    import pandas as pd

    for name in _PANDAS_READERS:
        fn = getattr(pd, name, None)
        if fn is None:
            continue

        def reader(path, *a, _fn=fn, **k):
            return _fn(_fuse_path(path), *a, **k)
        reader.__wrapped__ = fn
        reader.__doc__ = fn.__doc__
        _fuse_saved[("pd", name)] = fn
        setattr(pd, name, reader)
    for name in _PANDAS_WRITERS:
        fn = getattr(pd.DataFrame, name)

        def writer(self, path=None, *a, _fn=fn, **k):
            return _fn(self, _fuse_path(path), *a, **k)
        writer.__wrapped__ = fn
        _fuse_saved[("DataFrame", name)] = fn
        setattr(pd.DataFrame, name, writer)
    return True


def unmount_dbfs_fuse() -> None:
    import pandas as pd
    for (owner, name), fn in list(_fuse_saved.items()):
        setattr(pd if owner == "pd" else pd.DataFrame, name, fn)
    _fuse_saved.clear()


# ---------------------------------------------------------------- namespace

def _quiet_display(buf: Optional[list] = None, rows: int = 5):
    """``display`` that MATERIALISES what it is given (so a lazy plan that would fail
    in Databricks fails here too) but prints only a head."""
    def display(obj=None, *args, **kwargs):
        shown = obj
        if hasattr(obj, "toPandas") and hasattr(obj, "limit"):
            shown = obj.limit(1000).toPandas()
        elif hasattr(obj, "to_pandas") and hasattr(obj, "head"):
            shown = obj.head(1000).to_pandas()
        elif hasattr(obj, "toDebugString"):
            shown = obj.toDebugString
        elif hasattr(obj, "savefig"):
            return obj
        text = shown.head(rows).to_string() if hasattr(shown, "head") and hasattr(shown, "to_string") \
            else str(shown)[:2000]
        if buf is not None:
            buf.append(text)
        else:
            print(text)
    return display


def notebook_namespace(spark=None, lesson: Optional[str] = None, dataset_scale: float = 1.0,
                       install: bool = True, fuse: bool = True, quiet_display: bool = False,
                       module_name: str = "machine_learning") -> Dict[str, Any]:
    """The globals a course notebook sees after ``%run ./Includes/Classroom-Setup``."""
    from ..session import SparkSession
    from . import classroom as C
    from .dbutils import display, displayHTML

    spark = spark or SparkSession.builder.getOrCreate()
    spark.conf.set("com.databricks.training.module-name", module_name)  # SETUP:2
    cr = C.Classroom(spark, lesson=lesson, install=install, dataset_scale=dataset_scale)
    if fuse:
        mount_dbfs_fuse()
    disp = _quiet_display() if quiet_display else display
    tags = dbutils.notebook.getContext().tags()

    def getTag(tagName: str, defaultValue: str = None):  # noqa: N802 - UTIL:21
        return tags.get(tagName, defaultValue)

    def getDbrMajorAndMinorVersions():  # noqa: N802 - UTIL:33
        return (0, 0)

    def getLessonName():  # noqa: N802 - UTIL:69
        return cr.lesson

    def getDatabaseName(courseType, username, moduleName, lessonName):  # noqa: N802,N803 - UTIL:134
        return C.database_name(username, courseType)

    def createUserDatabase(courseType, username, moduleName, lessonName):  # noqa: N802,N803 - UTIL:144
        return C.create_user_database(spark, username, courseType, lessonName)

    def clearYourResults(passedOnly=True):  # noqa: N802,N803 - UTIL:168
        for k in [k for k, v in cr.test_results.items() if v["passed"] or not passedOnly]:
            del cr.test_results[k]

    def loadYourTestMap(path):  # noqa: N802 - UTIL:249
        return {k: v for k, v in cr.load_your_test_results(path).items()}

    def install_datasets(reinstall=False):  # SETUP:32
        from .datasets import install_datasets as inst
        inst(to_local(cr.datasets_dir), spark, reinstall=bool(reinstall), scale=dataset_scale)

    ns: Dict[str, Any] = dict(
        # Databricks-predefined names
        spark=spark, sc=spark.sparkContext, sql=spark.sql, table=spark.table,
        display=disp, displayHTML=(lambda html: None) if quiet_display else displayHTML, dbutils=dbutils,
        # Includes/Classroom-Setup.py:12-18
        username=cr.username, cleaned_username=cr.cleaned_username, userhome=cr.userhome,
        course_dir=cr.course_dir, datasets_dir=cr.datasets_dir, working_dir=cr.working_dir,
        path_exists=C.path_exists, install_datasets=install_datasets,
        init_mlflow_as_job=C.init_tracking_as_job, untilStreamIsReady=cr.until_stream_is_ready,
        # Includes/Class-Utility-Methods.py
        getTags=lambda: dict(tags), getTag=getTag, getDbrMajorAndMinorVersions=getDbrMajorAndMinorVersions,
        get_cloud=lambda: "local", getUsername=lambda: cr.username, getUserhome=lambda: cr.userhome,
        getModuleName=lambda: module_name, getLessonName=getLessonName,
        getCourseDir=lambda: cr.course_dir, getWorkingDir=lambda: cr.working_dir,
        getDatabaseName=getDatabaseName, createUserDatabase=createUserDatabase,
        testResults=cr.test_results, toHash=lambda value: C.to_hash(spark, value),
        clearYourResults=clearYourResults, validateYourSchema=cr.validate_your_schema,
        validateYourAnswer=cr.validate_your_answer, summarizeYourResults=cr.summarize_your_results,
        logYourTest=cr.log_your_test, loadYourTestResults=cr.load_your_test_results,
        loadYourTestMap=loadYourTestMap, pathExists=C.path_exists, deletePath=C.delete_path,
        deleteTables=lambda database: C.delete_tables(spark, database), allDone=cr.all_done,
        FILL_IN=C.FILL_IN, classroom=cr,
        __name__="__main__",
    )
    return ns


# ---------------------------------------------------------------- cells

_MAGIC = re.compile(r"^# MAGIC ?")


@dataclass
class Cell:
    index: int
    kind: str          # python | sql | run | md | pip | sh | fs | other
    code: str
    line: int          # 1-based line of the cell's first line in the file


def split_cells(source: str) -> List[Cell]:
    """Split Databricks notebook source into cells (``# COMMAND ----------``)."""
    out: List[Cell] = []
    line = 1
    for i, raw in enumerate(source.split("# COMMAND ----------")):
        start = line
        line += raw.count("\n")
        lines = [ln for ln in raw.split("\n") if not ln.startswith("# Databricks notebook source")]
        body = "\n".join(lines).strip("\n")
        if not body.strip():
            continue
        first = body.lstrip().split("\n", 1)[0]
        if first.startswith("# MAGIC"):
            text = "\n".join(_MAGIC.sub("", ln) for ln in body.strip().split("\n"))
            head = text.lstrip().split(None, 1)
            magic = head[0] if head else ""
            rest = head[1] if len(head) > 1 else ""
            kind = {"%sql": "sql", "%run": "run", "%md": "md", "%md-sandbox": "md", "%pip": "pip",
                    "%sh": "sh", "%fs": "fs"}.get(magic, "other")
            out.append(Cell(i, kind, rest.strip(), start))
            continue
        code_lines = [ln for ln in body.split("\n") if ln.strip() and not ln.strip().startswith("#")]
        if not code_lines:
            continue
        out.append(Cell(i, "python", body, start))
    return out


@dataclass
class CellResult:
    index: int
    kind: str
    line: int
    ok: bool
    seconds: float
    error: str = ""
    first_line: str = ""


@dataclass
class NotebookResult:
    path: str
    cells: List[CellResult] = field(default_factory=list)
    seconds: float = 0.0
    setup_error: str = ""

    @property
    def failed(self) -> List[CellResult]:
        return [c for c in self.cells if not c.ok]

    @property
    def n_ok(self) -> int:
        return sum(c.ok for c in self.cells)

    def to_json(self) -> Dict[str, Any]:
        d = asdict(self)
        d["n_ok"] = self.n_ok
        d["n_failed"] = len(self.failed)
        return d


def run_notebook(path: str, ns: Optional[Dict[str, Any]] = None, *, dataset_scale: float = 1.0,
                 lesson: Optional[str] = None, run_sql: bool = True, quiet: bool = True,
                 on_cell: Optional[Callable[[CellResult], None]] = None) -> NotebookResult:
    """Execute every cell of one notebook-source file in one namespace."""
    t0 = time.time()
    res = NotebookResult(path)
    if ns is None:
        try:
            ns = notebook_namespace(lesson=lesson or os.path.splitext(os.path.basename(path))[0],
                                    dataset_scale=dataset_scale, quiet_display=quiet)
        except Exception:  # noqa: BLE001
            res.setup_error = traceback.format_exc()
            res.seconds = time.time() - t0
            return res
    with open(path) as f:
        cells = split_cells(f.read())
    spark = ns["spark"]
    for c in cells:
        if c.kind in ("md", "pip", "run", "other") or (c.kind == "sql" and not run_sql):
            continue
        if c.kind in ("sh", "fs"):
            continue
        t1 = time.time()
        err = ""
        sink = io.StringIO()
        try:
            with redirect_stdout(sink) if quiet else _nullctx():
                if c.kind == "sql":
                    for stmt in [s for s in c.code.split(";") if s.strip()]:
                        ns["display"](spark.sql(stmt))
                else:
                    exec(compile(c.code, f"{os.path.basename(path)}:cell{c.index}@L{c.line}", "exec"), ns)
        except BaseException as e:  # noqa: BLE001 - SystemExit from dbutils.notebook.exit too
            if isinstance(e, KeyboardInterrupt):
                raise
            err = f"{type(e).__name__}: {e}\n" + "".join(traceback.format_exc().splitlines(True)[-6:])
        r = CellResult(c.index, c.kind, c.line, not err, time.time() - t1, err[:3000],
                       c.code.strip().split("\n", 1)[0][:120])
        res.cells.append(r)
        if on_cell is not None:
            on_cell(r)
    res.seconds = time.time() - t0
    return res


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def _fresh_root(base: str, nb_path: str) -> str:
    tag = re.sub(r"[^A-Za-z0-9]+", "_", os.path.splitext(os.path.basename(nb_path))[0]).strip("_")
    root = os.path.join(base, tag)
    os.makedirs(root, exist_ok=True)
    return root


def run_many(paths: List[str], workdir: str, dataset_scale: float = 0.05, verbose: bool = True
             ) -> List[NotebookResult]:
    """Run several notebooks in THIS process, each with its own DBFS root, tracking
    store, warehouse and database, like separate Databricks notebooks sharing a cluster."""
    from ..session import SparkSession
    out = []
    cwd = os.getcwd()
    env0 = {k: os.environ.get(k) for k in ("CDNAML_DBFS_ROOT", "CDNAML_TRACKING_URI")}
    try:
        _run_each(paths, workdir, dataset_scale, verbose, out, cwd, SparkSession)
    finally:
        _reset_process_state()
        for k, v in env0.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    return out


def _run_each(paths, workdir, dataset_scale, verbose, out, cwd, SparkSession):
    for p in paths:
        root = _fresh_root(workdir, p)
        _reset_process_state()   # before the env switch: open runs end in their own store
        os.environ["CDNAML_DBFS_ROOT"] = os.path.join(root, "dbfs")
        os.environ["CDNAML_TRACKING_URI"] = os.path.join(root, "mlruns")
        os.chdir(root)
        try:
            # a fresh session (own catalog, temp views, streams, conf) per notebook, like a notebook re-attach
            spark = SparkSession.builder.config("cdnaml.warehouse.dir",
                                                os.path.join(root, "spark-warehouse")).getOrCreate()
            try:
                ns = notebook_namespace(spark, lesson=os.path.splitext(os.path.basename(p))[0],
                                        dataset_scale=dataset_scale, quiet_display=True)
            except Exception:  # noqa: BLE001
                r = NotebookResult(p, setup_error=traceback.format_exc())
            else:
                r = run_notebook(p, ns)
        finally:
            unmount_dbfs_fuse()
            os.chdir(cwd)
        out.append(r)
        if verbose:
            print(f"=== {os.path.basename(p)}: {r.n_ok} ok, {len(r.failed)} failed, {r.seconds:.1f}s", flush=True)
            for c in r.failed:
                print(f"    cell {c.index} (L{c.line}) {c.first_line!r}\n      {c.error.splitlines()[0][:300]}",
                      flush=True)
            if r.setup_error:
                print("    setup: " + r.setup_error.splitlines()[-1], flush=True)


def _reset_process_state() -> None:
    """Forget per-notebook process state: tracking store, active runs, streams, catalog."""
    from ..session import SparkSession
    from ..tracking import fluent
    try:
        while fluent.active_run() is not None:
            fluent.end_run()
    except Exception:  # noqa: BLE001 - a notebook that left a run open in a deleted store
        pass
    fluent._global.update(uri=None, experiment_id=None, store=None, store_uri=None, stack=[])
    s = SparkSession.getActiveSession()
    if s is not None:
        for q in list(s.streams.active):
            q.stop()
        s.stop()


def main(argv: Optional[List[str]] = None) -> int:
    import argparse
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("notebooks", nargs="+")
    ap.add_argument("--scale", type=float, default=0.05)
    ap.add_argument("--workdir", default=None)
    ap.add_argument("--json", default=None)
    a = ap.parse_args(argv)
    os.environ.setdefault("MPLBACKEND", "Agg")
    import tempfile
    workdir = os.path.abspath(a.workdir or tempfile.mkdtemp(prefix="cdnaml_nb_"))
    import cdnaml.compat as compat
    compat.install()
    res = run_many([os.path.abspath(p) for p in a.notebooks], workdir, a.scale)
    if a.json:
        with open(a.json, "w") as f:
            json.dump([r.to_json() for r in res], f, indent=1)
    return 0 if all(not r.failed and not r.setup_error for r in res) else 1


if __name__ == "__main__":
    sys.exit(main())
