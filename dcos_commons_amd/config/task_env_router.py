"""Routes ``TASKCFG_ALL_*`` / ``TASKCFG_<POD>_*`` scheduler env into task environments.

Reference: sdk/.../config/TaskEnvRouter.java:26-133.
"""
from __future__ import annotations

import os
from typing import Dict, Mapping, Optional

from dcos_commons_amd.offer.taskdata.labels import to_env_name

TASKCFG_PREFIX = "TASKCFG_"
TASKCFG_GLOBAL_ENV_PREFIX = TASKCFG_PREFIX + "ALL_"


class TaskEnvRouter:
    def __init__(self, env: Optional[Mapping[str, str]] = None):
        env = os.environ if env is None else env
        self._env = {k: v for k, v in sorted(env.items()) if k.startswith(TASKCFG_PREFIX)}
        self._global: Dict[str, str] = {}
        self._pods: Dict[str, Dict[str, str]] = {}
        # routed config per pod type: a reference package routes ~300 TASKCFG_ variables and each
        # spec build asks once per pod type and task
        self._memo: Dict[str, Dict[str, str]] = {}

    def set_all_pods_env(self, key: str, value: str) -> "TaskEnvRouter":
        self._global[key] = value
        self._memo.clear()
        return self

    def set_pod_env(self, pod_type: str, key: str, value: str) -> "TaskEnvRouter":
        self._pods.setdefault(pod_type.lower(), {})[key] = value
        self._memo.clear()
        return self

    def get_config(self, pod_type: str) -> Dict[str, str]:
        hit = self._memo.get(pod_type)
        if hit is None:
            hit = self._memo[pod_type] = self._route(pod_type)
        return dict(hit)

    def _route(self, pod_type: str) -> Dict[str, str]:
        out = dict(sorted(self._global.items()))
        out.update(self._pods.get(pod_type.lower(), {}))
        pod_prefix = TASKCFG_PREFIX + to_env_name(pod_type) + "_"
        for k, v in self._env.items():
            if k.startswith(TASKCFG_GLOBAL_ENV_PREFIX):
                out[k[len(TASKCFG_GLOBAL_ENV_PREFIX):]] = v
            elif k.startswith(pod_prefix):
                out[k[len(pod_prefix):]] = v
        return dict(sorted(out.items()))
