"""Course harness helpers (Includes/Class-Utility-Methods.py,
Includes/Classroom-Setup.py).

``setup(lesson)`` resolves the same names the notebooks rely on —
``username``, ``cleaned_username``, ``userhome``, ``course_dir``,
``working_dir``, ``datasets_dir`` — creates the directories, installs the
synthetic datasets (H2) and the per-user database (H5).  The answer
validator hashes answers with Spark's ``abs(hash(value))`` exactly like the
course (UTIL:161-165) — our ``hash`` is bit-compatible Murmur3 — so the
expected constants in the labs check against this engine unchanged.
"""
from __future__ import annotations

import csv
import getpass
import os
import re
import time
from typing import Any, Dict, List, Optional

from .dbutils import dbutils, to_local

COURSE = "scalable-machine-learning-with-apache-spark"


class Classroom:
    def __init__(self, spark=None, course: str = COURSE, lesson: Optional[str] = None, root: Optional[str] = None,
                 install: bool = True, dataset_scale: float = 1.0):
        from ..session import SparkSession
        self.spark = spark or SparkSession.builder.getOrCreate()
        self.username = get_username(self.spark)
        # Classroom-Setup.py:13 -- the local part of the e-mail, lower-cased, non-alphanumerics -> "_"
        self.cleaned_username = re.sub(r"[^a-zA-Z0-9]", "_", self.username.lower().split("@")[0])
        self.userhome = f"dbfs:/user/{self.username}/dbacademy"
        self.course_dir = f"{self.userhome}/{course}"
        self.datasets_dir = f"{self.course_dir}/datasets"
        self.lesson = lesson or os.environ.get("CDNAML_LESSON", "lesson")
        clean_lesson = re.sub(r"[^a-zA-Z0-9]", "_", self.lesson).lower()
        self.working_dir = f"{self.course_dir}/{clean_lesson}"
        self.test_results: Dict[str, Dict[str, Any]] = {}
        if root is not None:
            os.environ["CDNAML_DBFS_ROOT"] = root
        dbutils.fs.mkdirs(self.working_dir)
        if install:
            from .datasets import install_datasets
            install_datasets(to_local(self.datasets_dir), self.spark, scale=dataset_scale)
        self.database = create_user_database(self.spark, self.cleaned_username, COURSE, self.lesson)
        self.spark.conf.set("com.databricks.training.module-name", "ml")

    # ------------------------------------------------------------ H3 answers
    def validate_your_answer(self, what: str, expected_hash: int, answer) -> bool:
        s = "null" if answer is None else "true" if answer is True else "false" if answer is False else str(answer)
        h = to_hash(self.spark, s)
        ok = h == int(expected_hash)
        self.test_results[what] = {"passed": ok, "answer": s, "hash": h}
        return ok

    validateYourAnswer = validate_your_answer

    def validate_your_schema(self, what: str, df, exp_column_name: str, exp_column_type: Optional[str] = None) -> bool:
        """Check that ``df`` has column ``exp_column_name`` (of type name ``exp_column_type`` when given, e.g.
        "double", "string", "vector"); records the outcome under "<what> contains <col>:<type>" (UTIL:175-194)."""
        key = f"{what} contains {exp_column_name}:{exp_column_type}"
        try:
            actual = df.schema[exp_column_name].dataType.typeName()
        except (KeyError, IndexError, AttributeError):
            self.test_results[what] = {"passed": False, "answer": "-not found-"}
            print(f"{key}: NOT found")
            return False
        ok = exp_column_type is None or actual == exp_column_type
        answer = "validated" if ok else f"{exp_column_name}:{actual}"
        self.test_results[key] = {"passed": ok, "answer": answer}
        print(f"{key}: validated" if ok else f"{key}: NOT matching ({answer})")
        return ok

    validateYourSchema = validate_your_schema

    def all_done(self, advertisements: Dict[str, tuple]) -> str:
        """Advertise the functions ("f"), variables ("v") and databases ("d") a setup cell defined (UTIL:297-351).

        ``advertisements[name] = (kind, signature_or_value, description)``; a name is hidden when the conf
        ``com.databricks.training.suppress.<name>`` is "true".  Returns the HTML (also sent to displayHTML)."""
        from html import escape

        from .dbutils import displayHTML
        shown = {k: v for k, v in advertisements.items()
                 if self.spark.conf.get(f"com.databricks.training.suppress.{k}", None) != "true"}
        parts = []
        for kind, title in (("f", "functions were defined"), ("v", "variables were defined"),
                            ("d", "database were created")):
            items = [(k, v) for k, v in shown.items() if v[0] == kind]
            if not items:
                continue
            lis = []
            for k, v in items:
                if kind == "f":
                    body = f"<b>{escape(k)}</b>(<i>{escape(str(v[1]))}</i>)"
                elif kind == "v":
                    body = f"<b>{escape(k)}</b>: <i>{escape(str(v[1]))}</i>"
                else:
                    body = f"Now using the database identified by <b>{escape(k)}</b>: <i>{escape(str(v[1]))}</i>"
                lis.append(f"<li>{body}<div>{escape(str(v[2]))}</div></li>")
            parts.append(f"The following {title} for you:<ul>{''.join(lis)}</ul>")
        html = "".join(parts) + "All done!"
        displayHTML(html)
        return html

    allDone = all_done

    def summarize_your_results(self) -> str:
        rows = [f"<tr><th>{k}</th><td>{'passed' if v['passed'] else 'FAILED'}</td></tr>"
                for k, v in self.test_results.items()]
        return "<table>" + "".join(rows) + "</table>"

    summarizeYourResults = summarize_your_results

    def log_your_test(self, path: str, name: str, value) -> None:
        p = to_local(path)
        os.makedirs(os.path.dirname(os.path.abspath(p)), exist_ok=True)
        with open(p, "a", newline="") as f:
            csv.writer(f).writerow([name, value])

    logYourTest = log_your_test

    def load_your_test_results(self, path: str) -> Dict[str, str]:
        with open(to_local(path)) as f:
            return {r[0]: r[1] for r in csv.reader(f) if r}

    loadYourTestResults = load_your_test_results

    def clear_your_results(self):
        self.test_results.clear()

    clearYourResults = clear_your_results

    # ------------------------------------------------------------ H10 streams
    def until_stream_is_ready(self, name: str, progressions: int = 3, timeout: float = 60.0):
        """Busy-wait until the named query reports progress (SETUP:96-110)."""
        t0 = time.time()
        while True:
            qs = [q for q in self.spark.streams.active if q.name == name]
            if qs and len(qs[0].recentProgress) >= progressions:
                return qs[0]
            if time.time() - t0 > timeout:
                raise TimeoutError(f"stream {name!r} made no progress in {timeout}s")
            time.sleep(0.2)

    untilStreamIsReady = until_stream_is_ready

    # ------------------------------------------------------------ H11 reset
    def reset(self):
        dbutils.fs.rm(self.course_dir, True)

    def names(self) -> Dict[str, str]:
        return {"username": self.username, "cleaned_username": self.cleaned_username, "userhome": self.userhome,
                "course_dir": self.course_dir, "datasets_dir": self.datasets_dir, "working_dir": self.working_dir}


def get_username(spark=None) -> str:
    """``SELECT current_user()`` (UTIL:51-60); env ``CDNAML_USER`` overrides."""
    u = os.environ.get("CDNAML_USER")
    if u:
        return u
    try:
        u = getpass.getuser()
    except Exception:  # noqa: BLE001
        u = "user"
    return f"{u}@cdnaml.local"


def to_hash(spark, value) -> int:
    """``abs(hash(str(value)))`` cast to int, computed by the engine (UTIL:161-165)."""
    from ..sql import functions as F
    df = spark.createDataFrame([(str(value),)], ["value"])
    return int(df.select(F.abs(F.hash(F.col("value"))).cast("int").alias("h")).first().h)


def database_name(username: str, course: str) -> str:
    """Per-user database name (UTIL:134-142)."""
    return re.sub(r"[^a-zA-Z0-9]", "_", f"{username}_{course[:12]}").lower()


def create_user_database(spark, username: str, course: str, lesson: str) -> str:
    """Per-user database (UTIL:134-150)."""
    name = database_name(username, course)
    spark.sql(f"CREATE DATABASE IF NOT EXISTS {name}")
    spark.sql(f"USE {name}")
    return name


def delete_tables(spark, database: str):
    spark.sql(f"DROP DATABASE IF EXISTS {database} CASCADE")


def path_exists(path: str) -> bool:
    return os.path.exists(to_local(path))


def delete_path(path: str) -> bool:
    return dbutils.fs.rm(path, True)


def platform_info() -> Dict[str, Any]:
    """Runtime / device introspection (H8): ROCm + GPU details instead of DBR tags."""
    import torch
    info = {"runtime": f"cdnaml {__import__('cdnaml').__version__}", "torch": torch.__version__,
            "hip": getattr(torch.version, "hip", None), "gpus": 0, "devices": []}
    if torch.cuda.is_available():
        info["gpus"] = torch.cuda.device_count()
        info["devices"] = [torch.cuda.get_device_properties(i).name for i in range(info["gpus"])]
    return info


def init_tracking_as_job(job_id: Optional[str] = None):
    """H9: when run as a job, route experiments to ``/Curriculum/Test Results/Experiments/{jobId}``."""
    from .. import tracking
    jid = job_id or dbutils.notebook.getContext().tags().get("jobId")
    if jid:
        return tracking.set_experiment(f"/Curriculum/Test Results/Experiments/{jid}")
    return None


class FILL_IN:  # noqa: N801 - course placeholder (UTIL:356-363)
    VALUE = None
    LIST = []
    SCHEMA = None
    ROW = None
    INT = 0
    DATAFRAME = None
