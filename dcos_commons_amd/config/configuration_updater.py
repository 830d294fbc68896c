"""Configuration update on scheduler start.

Reference: sdk/.../config/DefaultConfigurationUpdater.java:159-467. Loads the current target,
logs a unified diff, runs the validators (fatal errors stop the scheduler), stores and targets
the new config if it changed, re-labels tasks whose pod spec is effectively unchanged (count,
placement, role and allow-decommission are ignored) and garbage-collects unreferenced configs.
"""
from __future__ import annotations

import difflib
import logging
from dataclasses import replace
from typing import List, Optional

from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.offer.taskdata.labels import TaskException, TaskLabelReader, TaskLabelWriter
from dcos_commons_amd.specification.specs import DEFAULT_SERVICE_USER, ResourceSet, ResourceSpec
from dcos_commons_amd.state.config_store import ConfigStoreException
from dcos_commons_amd.storage.persister import Reason

LOGGER = logging.getLogger(__name__)


class UpdateResult:
    def __init__(self, target_id, errors):
        self.target_id = target_id
        self.errors = list(errors)


def _filter_irrelevant(pod):
    dummy = "dummy-role"
    tasks = []
    for t in pod.tasks:
        rs = t.resource_set
        # Every resource (ports included) is reduced to a plain DefaultResourceSpec with a dummy role,
        # as DefaultResourceSpec.newBuilder(copy).role(dummy) does in the reference.
        resources = tuple(ResourceSpec(name=r.name, value=r.value, role=dummy, principal=r.principal,
                                       pre_reserved_role=r.pre_reserved_role) for r in rs.resources)
        vols = tuple(replace(v, role=dummy, pre_reserved_role="*") for v in rs.volumes)
        new_rs = ResourceSet(id=rs.id, resources=resources, volumes=vols, role=dummy, principal=rs.principal,
                             pre_reserved_role=None)
        tasks.append(replace(t, resource_set=new_rs))
    return replace(pod, count=0, placement_rule=None, allow_decommission=False, tasks=tuple(tasks))


def pods_match(a, b) -> bool:
    if a == b:
        return True
    return _filter_irrelevant(a) == _filter_irrelevant(b)


class DefaultConfigurationUpdater:
    def __init__(self, state_store, config_store, validators, namespace: Optional[str] = None):
        self.state_store = state_store
        self.config_store = config_store
        self.validators = list(validators)
        self.logger = logging.getLogger(__name__ + (f"({namespace})" if namespace else ""))

    def update_configuration(self, candidate) -> UpdateResult:
        try:
            target_id = self.config_store.get_target_config()
        except ConfigStoreException:
            target_id = None
        target = self.config_store.fetch(target_id) if target_id is not None else None
        errors = []
        if target is not None:
            self._print_diff(target, target_id, candidate)
        target = self._fix_user(target)
        for v in self.validators:
            errors.extend(v(target, candidate))
        if errors:
            lines = "\n".join(f"{i + 1}: {e}" for i, e in enumerate(errors))
            self.logger.warning("New configuration failed validation against current target configuration %s, "
                                "with %d errors across %d validators:\n%s", target_id, len(errors),
                                len(self.validators), lines)
            for e in errors:
                if e.is_fatal():
                    raise ConfigStoreException(
                        Reason.LOGIC_ERROR, f"FATAL ERROR with Configuration Update, stopping scheduler.\nError:{e}")
            if target is None:
                raise ConfigStoreException(
                    Reason.LOGIC_ERROR,
                    "Configuration failed validation without any prior target configuration available for "
                    f"fallback. Initial launch with invalid configuration? {len(errors)} Errors: {lines}")
        elif target is None or target != candidate:
            old_id = target_id
            target_id = self.config_store.store(candidate)
            self.logger.info("Updating target configuration: Prior target configuration '%s' is different from "
                             "new configuration '%s'.", old_id, target_id)
            target = candidate
            self.config_store.set_target_config(target_id)
        else:
            self.logger.info("No changes detected between current target configuration '%s' and new "
                             "configuration. Leaving current configuration as the target.", target_id)
        self._cleanup(target, target_id)
        return UpdateResult(target_id, errors)

    @staticmethod
    def _fix_user(target):
        if target is None:
            return None
        pods = tuple(p if p.user else replace(p, user=DEFAULT_SERVICE_USER) for p in target.pods)
        return replace(target, user=target.user or DEFAULT_SERVICE_USER, pods=pods)

    def _print_diff(self, old, old_id, new) -> None:
        if not self.logger.isEnabledFor(logging.INFO):
            return  # the diff of two rendered specs is the costliest part of a restart's update
        try:
            diff = difflib.unified_diff(old.to_json_string().splitlines(), new.to_json_string().splitlines(),
                                        "ServiceSpec.old", "ServiceSpec.new", n=2, lineterm="")
            text = "\n".join(diff)
            if text:
                self.logger.info("Difference between configs:\n%s", text)
        except Exception:  # noqa: BLE001
            self.logger.exception("Unable to diff target config %s against the new config", old_id)

    def _needs_config_update(self, info: P.TaskInfo, target, task_config, memo: Optional[dict] = None) -> bool:
        """``memo`` (one per cleanup pass): the spec and pod comparisons depend only on the two
        configs and the pod type, so the tasks of a pod type are compared once, not per task
        (a reference hdfs spec compares ~320-variable environments)."""
        memo = {} if memo is None else memo
        same = memo.get(id(task_config))
        if same is None:
            same = memo[id(task_config)] = target == task_config
        if same:
            return False
        try:
            r = TaskLabelReader(info)
            pod_type = r.get_type()
            perm_failed = r.is_permanently_failed()
        except TaskException:
            return True
        if perm_failed:
            return False
        key = (id(task_config), pod_type)
        match = memo.get(key)
        if match is None:
            tp, op = target.pod(pod_type), task_config.pod(pod_type)
            match = memo[key] = tp is not None and op is not None and pods_match(tp, op)
        return not match

    def _cleanup(self, target, target_id) -> None:
        to_update: List[P.TaskInfo] = []
        needed = {target_id}
        memo: dict = {}
        for info in self.state_store.fetch_tasks_shared():     # updated on copies
            try:
                cid = TaskLabelReader(info).get_target_configuration()
            except (TaskException, ValueError):
                continue
            if cid == target_id:
                continue
            try:
                task_config = self.config_store.fetch(cid)
            except ConfigStoreException:
                needed.add(cid)
                continue
            if not self._needs_config_update(info, target, task_config, memo):
                c = P.TaskInfo()
                c.CopyFrom(info)
                TaskLabelWriter(c).set_target_configuration(target_id).apply()
                to_update.append(c)
            else:
                needed.add(cid)
        if to_update:
            self.logger.info("Updating %d tasks in StateStore with target configuration ID %s", len(to_update),
                             target_id)
            self.state_store.store_tasks(to_update)
        for cid in self.config_store.list():
            try:
                self.config_store.fetch(cid)
            except ConfigStoreException:
                needed.add(cid)
        for cid in self.config_store.list():
            if cid not in needed:
                self.config_store.clear(cid)
