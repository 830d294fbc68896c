"""Write-ahead recording of launches.

Reference: sdk/.../state/PersistentLaunchRecorder.java:32-212. Every ``StoreTaskInfoRecommendation``
is persisted *before* the ACCEPT is sent (empty-TaskID entries first), together with a synthetic
``TASK_STAGING`` status for real launches; tasks sharing a resource set with the launched task get
the new resources copied onto their stored TaskInfo.

Addition: a launch whose task resources (its own resource set; the executor's resources are not
considered) reference only reservations that no stored task of its pod instance referenced before
this batch created its whole footprint (first launch or permanent replace). Its stored TaskInfo
carries ``launch_new_footprint=true``; an in-place relaunch that reuses existing reservations or
volumes never does.

A pod's first footprint reserves every resource set of the pod, including those of tasks that
only launch later (sidecars started by a plan, reference OfferEvaluator.java:411-536), and stores a
TaskInfo (empty TaskID) for each of them. So the first launch of such a task reuses reservations
that exist and is never labelled: a lost ACCEPT there is a transient LOST relaunched in place
(``test_lost_accept_of_a_new_resource_set_next_to_a_running_executor_is_relaunched``).
"""
from __future__ import annotations

import logging
from typing import Dict, Optional

from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.offer import task_utils
from dcos_commons_amd.offer.recommendations import StoreTaskInfoRecommendation
from dcos_commons_amd.offer.resources import get_all_resources, get_resource_ids
from dcos_commons_amd.offer.taskdata.labels import TaskException, TaskLabelReader, TaskLabelWriter
from dcos_commons_amd.specification.specs import PodInstance


class PersistentLaunchRecorder:
    def __init__(self, state_store, service_spec, namespace: Optional[str] = None):
        self.state_store = state_store
        self.service_spec = service_spec
        self.logger = logging.getLogger(__name__ + (f"({namespace})" if namespace else ""))

    def record(self, recommendations) -> None:
        stores = [r for r in recommendations if isinstance(r, StoreTaskInfoRecommendation)]
        stores.sort(key=lambda r: len(r.task_info.task_id.value))
        infos = [rec.state_store_task_info() for rec in stores]
        # reservations the pod instances of this batch referenced before any of it is written
        prior_ids = {}
        for info in infos:
            if info.task_id.value == "":
                continue
            pi = self._pod_instance(info)
            if pi is not None and pi.name not in prior_ids:
                prior_ids[pi.name] = self._stored_resource_ids(pi)
        # the batch is applied to working copies in recommendation order, then written at once:
        # TaskInfos in one ``store_tasks`` (the StateStore splits it at 1 MB), statuses after them.
        # A peer sharing a resource set is rewritten once with the last resources of the batch
        # instead of once per launched task (a cassandra node: 13 tasks on one set), and only if
        # they changed.
        working: Dict[str, P.TaskInfo] = {}
        fetched: Dict[str, Optional[P.TaskInfo]] = {}
        statuses = []
        for info in infos:
            status = None
            pi = self._pod_instance(info)
            if info.task_id.value != "":
                status = P.TaskStatus(state=P.TASK_STAGING)
                status.task_id.CopyFrom(info.task_id)
                if info.HasField("executor"):
                    status.executor_id.CopyFrom(info.executor.executor_id)
                ids = get_resource_ids(info.resources)
                new = bool(ids) and pi is not None and not (set(ids) & prior_ids.get(pi.name, set()))
                TaskLabelWriter(info).set_launch_new_footprint(new).apply()
            if pi is not None:
                self._update_resource_set_peers(pi, info, working, fetched)
            working.pop(info.name, None)
            working[info.name] = info
            if status is not None:
                statuses.append((info.name, status))
        if working:
            # TaskInfos and their STAGING statuses in one transaction when they fit one batch
            self.state_store.store_tasks(list(working.values()), statuses)
        else:
            for name, status in statuses:
                self.state_store.store_status(name, status)

    def _pod_instance(self, info: P.TaskInfo) -> Optional[PodInstance]:
        try:
            pod = task_utils.get_pod_spec(self.service_spec, info)
            return PodInstance(pod, TaskLabelReader(info).get_index()) if pod is not None else None
        except (TaskException, ValueError):
            return None

    def _stored_resource_ids(self, pi: PodInstance) -> set:
        out = set()
        for t in pi.pod.tasks:
            stored = self.state_store.fetch_task_shared(f"{pi.name}-{t.name}")
            if stored is not None:
                out.update(get_resource_ids(get_all_resources(stored)))
        return out

    def _update_resource_set_peers(self, pi: PodInstance, info: P.TaskInfo,
                                   working: Optional[Dict[str, P.TaskInfo]] = None,
                                   fetched: Optional[Dict[str, Optional[P.TaskInfo]]] = None) -> None:
        """Copies ``info``'s task and executor resources onto the other tasks of its resource set
        (PersistentLaunchRecorder.updateResourcesWithinResourceSet): into ``working`` during a
        batch, or straight to the StateStore without one. ``fetched`` memoizes the stored peers
        read during the batch, so a set of N tasks is read N times, not N squared."""
        spec = task_utils.get_task_spec(pi, info.name)
        if spec is None:
            return
        standalone = working is None
        if standalone:
            working = {}
        if fetched is None:
            fetched = {}
        has_executor = info.HasField("executor")
        for t in pi.pod.tasks:
            if t.name == spec.name or t.resource_set != spec.resource_set:
                continue
            name = f"{pi.name}-{t.name}"
            peer = working.get(name)
            if peer is None:
                if name not in fetched:
                    fetched[name] = self.state_store.fetch_task_shared(name)
                stored = fetched[name]
                if stored is None:
                    continue
                if list(stored.resources) == list(info.resources) and (
                        not has_executor or list(stored.executor.resources) == list(info.executor.resources)):
                    continue  # already what this launch would write
                peer = P.TaskInfo()      # the stored one is shared with the state store's readers
                peer.CopyFrom(stored)
            del peer.resources[:]
            peer.resources.extend(info.resources)
            if has_executor:
                del peer.executor.resources[:]
                peer.executor.resources.extend(info.executor.resources)
            working[name] = peer
        if standalone and working:
            self.state_store.store_tasks(list(working.values()))
