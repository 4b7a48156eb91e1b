"""``dbutils`` equivalents: file-system helpers, widgets,
notebook context, plus ``display`` / ``displayHTML``.

``dbfs:/…`` paths map onto a local root (``CDNAML_DBFS_ROOT``, default
``./dbfs``) so course code that mixes ``dbfs:/`` URIs and ``/dbfs/`` POSIX
paths keeps working.
"""
from __future__ import annotations

import os
import shutil
from typing import Dict, List, Optional


def dbfs_root() -> str:
    return os.path.abspath(os.environ.get("CDNAML_DBFS_ROOT", "dbfs"))


def to_local(path) -> str:
    """The ONE DBFS resolver used by every reader, writer, Delta table, stream,
    catalog location, model path and ``dbutils.fs`` call.

    ``dbfs:/x``, ``dbfs:x``, ``/dbfs/x``, ``file:/dbfs/x`` and ``file:///dbfs/x``
    all resolve to ``<dbfs_root>/x`` (the FUSE mount of ``Includes/Reset.py:11`` and
    the ``.replace("dbfs:/", "/dbfs/")`` idiom of ``ML 05:69`` / ``ML 12:34``);
    ``file:/x`` / ``file:///x`` -> ``/x``; anything else is a host path.  A ``dbfs:``
    URI never resolves outside the DBFS root: ``..`` components are rejected."""
    if not isinstance(path, str):
        path = os.fspath(path)
    if path.startswith("file:"):
        rest = path[len("file:"):]
        local = "/" + rest.lstrip("/") if rest.startswith("/") else rest
        if local == "/dbfs" or local.startswith("/dbfs/"):
            return _under_root(local[len("/dbfs"):])
        return local
    if path.startswith("dbfs:"):
        return _under_root(path[len("dbfs:"):])
    if path == "/dbfs" or path.startswith("/dbfs/"):
        return _under_root(path[len("/dbfs"):])
    return path


def _under_root(rel: str) -> str:
    root = dbfs_root()
    rel = rel.lstrip("/")
    if not rel:
        return root
    full = os.path.normpath(os.path.join(root, rel))
    if full != root and not full.startswith(root + os.sep):
        raise ValueError(f"DBFS path escapes the DBFS root: {rel!r}")
    if rel.endswith("/"):
        full += "/"
    return full


class FileInfo:
    def __init__(self, path: str, name: str, size: int, modificationTime: int):
        self.path = path
        self.name = name
        self.size = size
        self.modificationTime = modificationTime

    def isDir(self):
        return self.name.endswith("/")

    def isFile(self):
        return not self.isDir()

    def __repr__(self):
        return f"FileInfo(path='{self.path}', name='{self.name}', size={self.size})"

    def __iter__(self):
        return iter((self.path, self.name, self.size, self.modificationTime))


class _FS:
    def ls(self, path: str) -> List[FileInfo]:
        p = to_local(path)
        if not os.path.exists(p):
            raise FileNotFoundError(f"java.io.FileNotFoundException: File {path} does not exist.")
        if os.path.isfile(p):
            st = os.stat(p)
            return [FileInfo(path, os.path.basename(p), st.st_size, int(st.st_mtime * 1000))]
        out = []
        for name in sorted(os.listdir(p)):
            full = os.path.join(p, name)
            st = os.stat(full)
            d = os.path.isdir(full)
            out.append(FileInfo(path.rstrip("/") + "/" + name + ("/" if d else ""), name + ("/" if d else ""),
                                0 if d else st.st_size, int(st.st_mtime * 1000)))
        return out

    def rm(self, path: str, recurse: bool = False) -> bool:
        p = to_local(path)
        if not os.path.exists(p):
            return False
        if os.path.isdir(p):
            if not recurse and os.listdir(p):
                raise IOError(f"{path} is a non-empty directory; use recurse=True")
            shutil.rmtree(p)
        else:
            os.remove(p)
        return True

    def mkdirs(self, path: str) -> bool:
        os.makedirs(to_local(path), exist_ok=True)
        return True

    def cp(self, src: str, dst: str, recurse: bool = False) -> bool:
        s, d = to_local(src), to_local(dst)
        if os.path.isdir(s):
            if not recurse:
                raise IOError(f"{src} is a directory; use recurse=True")
            shutil.copytree(s, d, dirs_exist_ok=True)
        else:
            os.makedirs(os.path.dirname(os.path.abspath(d)), exist_ok=True)
            shutil.copy2(s, d)
        return True

    def mv(self, src: str, dst: str, recurse: bool = False) -> bool:
        shutil.move(to_local(src), to_local(dst))
        return True

    def head(self, path: str, maxBytes: int = 65536) -> str:
        with open(to_local(path), "rb") as f:
            return f.read(maxBytes).decode("utf-8", errors="replace")

    def put(self, path: str, contents: str, overwrite: bool = False) -> bool:
        p = to_local(path)
        if os.path.exists(p) and not overwrite:
            raise FileExistsError(f"{path} already exists (overwrite=False)")
        os.makedirs(os.path.dirname(os.path.abspath(p)), exist_ok=True)
        with open(p, "w") as f:
            f.write(contents)
        return True


class _Widgets:
    def __init__(self):
        self._v: Dict[str, str] = {}

    def text(self, name: str, defaultValue: str = "", label: Optional[str] = None):
        self._v.setdefault(name, os.environ.get(f"CDNAML_WIDGET_{name.upper()}", defaultValue))

    def dropdown(self, name, defaultValue, choices, label=None):
        self.text(name, defaultValue)

    combobox = dropdown
    multiselect = dropdown

    def get(self, name: str) -> str:
        if name not in self._v:
            raise KeyError(f"InputWidgetNotDefined: No input widget named {name} is defined")
        return self._v[name]

    def getArgument(self, name, default=None):
        return self._v.get(name, default)

    def remove(self, name):
        self._v.pop(name, None)

    def removeAll(self):
        self._v.clear()


class _Notebook:
    def __init__(self):
        self._tags = {"jobId": os.environ.get("CDNAML_JOB_ID", ""), "clusterId": "cdnaml-local",
                      "notebookPath": os.environ.get("CDNAML_NOTEBOOK_PATH", "")}

    def getContext(self):
        return self

    def tags(self):
        return dict(self._tags)

    def exit(self, value: str):
        raise SystemExit(value)


class DBUtils:
    def __init__(self):
        self.fs = _FS()
        self.widgets = _Widgets()
        self.notebook = _Notebook()


dbutils = DBUtils()


def display(obj, *args, **kwargs):
    """Databricks ``display``: show a DataFrame (first 1000 rows), a pandas-API frame,
    a model's tree (``toDebugString``) or a matplotlib figure."""
    if hasattr(obj, "show") and hasattr(obj, "toPandas"):
        print(obj.limit(1000).toPandas().to_string(max_rows=50))
    elif hasattr(obj, "to_pandas"):
        print(obj.head(1000).to_pandas().to_string(max_rows=50))
    elif hasattr(obj, "toDebugString"):
        print(obj.toDebugString)
    elif hasattr(obj, "savefig"):
        return obj
    else:
        print(obj)


def displayHTML(html: str):
    print(html)
