"""``MlflowClient``-compatible client over the file store.

Stage transitions with ``archive_existing_versions`` (ML 05 - MLflow Model
Registry.py:171-175,293-298), descriptions, ``search_model_versions("name =
'…'")``, delete (a version must be archived first, ML 05:304).
"""
from __future__ import annotations

import os
import re
import shutil
from typing import List, Optional

from . import fluent
from .entities import ModelVersion, TrackingException
from .store import FileStore

_STAGES = {"none": "None", "staging": "Staging", "production": "Production", "archived": "Archived"}


class MlflowClient:
    def __init__(self, tracking_uri: Optional[str] = None, registry_uri: Optional[str] = None):
        self._uri = tracking_uri

    @property
    def _store(self) -> FileStore:
        if self._uri:
            return FileStore(self._uri)
        return fluent._store()

    # ------------------------------------------------------------- experiments
    def list_experiments(self, view_type="ACTIVE_ONLY", max_results=None):
        return self._store.list_experiments(view_type)[:max_results] if max_results else \
            self._store.list_experiments(view_type)

    search_experiments = list_experiments

    def get_experiment(self, experiment_id):
        return self._store.get_experiment(experiment_id)

    def get_experiment_by_name(self, name):
        return self._store.get_experiment_by_name(name)

    def create_experiment(self, name, artifact_location=None, tags=None):
        return self._store.create_experiment(name, artifact_location, tags)

    def delete_experiment(self, experiment_id):
        self._store.delete_experiment(experiment_id)

    def set_experiment_tag(self, experiment_id, key, value):
        self._store.set_experiment_tag(experiment_id, key, value)

    # ------------------------------------------------------------- runs
    def create_run(self, experiment_id, start_time=None, tags=None, run_name=None):
        return self._store.create_run(experiment_id, fluent._user(), start_time, tags, run_name)

    def get_run(self, run_id):
        return self._store.get_run(run_id)

    def search_runs(self, experiment_ids, filter_string="", run_view_type=None, max_results=1000, order_by=None,
                    page_token=None):
        return fluent._search(experiment_ids, filter_string, order_by, max_results)

    def list_run_infos(self, experiment_id, run_view_type=None, max_results=None, order_by=None):
        return [r.info for r in fluent._search([experiment_id], "", order_by, max_results)]

    def log_param(self, run_id, key, value):
        self._store.log_param(run_id, key, value)

    def log_metric(self, run_id, key, value, timestamp=None, step=None):
        self._store.log_metric(run_id, key, value, timestamp, step or 0)

    def set_tag(self, run_id, key, value):
        self._store.set_tag(run_id, key, value)

    def delete_tag(self, run_id, key):
        self._store.delete_tag(run_id, key)

    def log_artifact(self, run_id, local_path, artifact_path=None):
        dst = os.path.join(self._store.artifact_dir(run_id), artifact_path or "")
        os.makedirs(dst, exist_ok=True)
        shutil.copy2(local_path, os.path.join(dst, os.path.basename(local_path)))

    def set_terminated(self, run_id, status="FINISHED", end_time=None):
        import time
        self._store.update_run(run_id, status=status, end_time=end_time or int(time.time() * 1000))

    def delete_run(self, run_id):
        self._store.delete_run(run_id)

    def get_metric_history(self, run_id, key):
        return self._store.get_metric_history(run_id, key)

    def list_artifacts(self, run_id, path=None):
        base = os.path.join(self._store.artifact_dir(run_id), path or "")

        class FileInfo:
            def __init__(self, p, is_dir, size):
                self.path, self.is_dir, self.file_size = p, is_dir, size

            def __repr__(self):
                return f"<FileInfo: path='{self.path}', is_dir={self.is_dir}>"
        if not os.path.isdir(base):
            return []
        return [FileInfo(os.path.join(path, f) if path else f, os.path.isdir(os.path.join(base, f)),
                         None if os.path.isdir(os.path.join(base, f)) else os.path.getsize(os.path.join(base, f)))
                for f in sorted(os.listdir(base))]

    def download_artifacts(self, run_id, path, dst_path=None):
        src = os.path.join(self._store.artifact_dir(run_id), path)
        if dst_path is None:
            return src
        dst = os.path.join(dst_path, os.path.basename(path))
        if os.path.isdir(src):
            shutil.copytree(src, dst, dirs_exist_ok=True)
        else:
            os.makedirs(dst_path, exist_ok=True)
            shutil.copy2(src, dst)
        return dst

    # ------------------------------------------------------------- registry
    def create_registered_model(self, name, tags=None, description=None):
        return self._store.create_registered_model(name, tags, description)

    def get_registered_model(self, name):
        return self._store.get_registered_model(name)

    def update_registered_model(self, name, description=None):
        return self._store.update_registered_model(name, description)

    def rename_registered_model(self, name, new_name):
        self._store.rename_registered_model(name, new_name)

    def delete_registered_model(self, name):
        self._store.delete_registered_model(name)

    def list_registered_models(self, max_results=100):
        return self._store.list_registered_models()[:max_results]

    search_registered_models = list_registered_models

    def create_model_version(self, name, source, run_id=None, tags=None, description=None):
        return self._store.create_model_version(name, source, run_id, tags, description)

    def get_model_version(self, name, version) -> ModelVersion:
        return self._store.get_model_version(name, version)

    def update_model_version(self, name, version, description=None):
        return self._store.update_model_version(name, version, description=description)

    def transition_model_version_stage(self, name, version, stage, archive_existing_versions=False):
        st = _STAGES.get(str(stage).lower())
        if st is None:
            raise TrackingException(f"Invalid Model Version stage: {stage}. Value must be one of None, Staging, "
                                    f"Production, Archived.")
        if archive_existing_versions and st in ("Staging", "Production"):
            for v in self._store.search_model_versions_for(name):
                if v.current_stage == st and int(v.version) != int(version):
                    self._store.update_model_version(name, v.version, stage="Archived")
        return self._store.update_model_version(name, version, stage=st)

    def delete_model_version(self, name, version):
        mv = self._store.get_model_version(name, version)
        if mv.current_stage in ("Staging", "Production"):
            raise TrackingException(f"Model version {version} of '{name}' is in stage {mv.current_stage}; transition "
                                    f"it to 'Archived' or 'None' before deleting.")
        self._store.delete_model_version(name, version)

    def get_latest_versions(self, name, stages=None) -> List[ModelVersion]:
        vs = self._store.search_model_versions_for(name)
        latest = {}
        for v in vs:
            latest[v.current_stage] = v
        if stages:
            return [latest[s] for s in (_STAGES.get(x.lower(), x) for x in stages) if s in latest]
        return list(latest.values())

    def search_model_versions(self, filter_string: str = "", max_results=None):
        m = re.match(r"\s*name\s*=\s*['\"]([^'\"]+)['\"]\s*$", filter_string or "")
        names = [m.group(1)] if m else [r.name for r in self._store.list_registered_models()]
        out = []
        for n in names:
            out.extend(self._store.search_model_versions_for(n))
        rm = re.match(r"\s*run_id\s*=\s*['\"]([^'\"]+)['\"]\s*$", filter_string or "")
        if rm:
            out = [v for r in self._store.list_registered_models() for v in
                   self._store.search_model_versions_for(r.name) if v.run_id == rm.group(1)]
        return out[:max_results] if max_results else out

    def get_model_version_download_uri(self, name, version):
        return self._store.get_model_version(name, version).source
