"""TaskID / ExecutorID construction and parsing.

Reference: sdk/.../offer/CommonIdUtils.java. IDs are
``<sanitized-service>__<name>__<uuid>`` where ``/`` in the service name becomes ``.``.
"""
from __future__ import annotations

from typing import Optional

from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.offer.taskdata.labels import TaskException
from dcos_commons_amd.utils import ids

NAME_ID_DELIM = "__"


def to_sanitized_service_name(service_name: str) -> str:
    return service_name.strip("/").replace("/", ".")


def _to_id_string(service_name: str, item_name: str) -> str:
    if NAME_ID_DELIM in service_name:
        raise ValueError(f"Service cannot contain delimiter '{NAME_ID_DELIM}': {service_name}")
    if NAME_ID_DELIM in item_name:
        raise ValueError(f"Name cannot contain delimiter '{NAME_ID_DELIM}': {item_name}")
    return f"{to_sanitized_service_name(service_name)}{NAME_ID_DELIM}{item_name}{NAME_ID_DELIM}{ids.uuid4_str()}"


def to_task_id(service_name: str, task_name: str) -> P.TaskID:
    return P.TaskID(value=_to_id_string(service_name, task_name))


def to_executor_id(service_name: str, executor_name: str) -> P.ExecutorID:
    return P.ExecutorID(value=_to_id_string(service_name, executor_name))


def _seek_back_from(id_: str, end: int) -> str:
    begin = id_.rfind(NAME_ID_DELIM, 0, end)
    if begin == -1:
        return id_[:end]
    return id_[begin + len(NAME_ID_DELIM):end]


def _extract(id_: str, service_name: bool) -> Optional[str]:
    last = id_.rfind(NAME_ID_DELIM)
    if last == -1:
        raise TaskException(
            f"ID '{id_}' is malformed. Expected '{NAME_ID_DELIM}' to extract name from ID. "
            "IDs should be generated with CommonIdUtils.")
    if not service_name:
        return _seek_back_from(id_, last)
    second = id_.rfind(NAME_ID_DELIM, 0, last)
    if second == -1:
        return None
    return _seek_back_from(id_, second)


def to_task_name(task_id) -> str:
    value = task_id.value if hasattr(task_id, "value") else task_id
    return _extract(value, False)


def to_executor_name(executor_id) -> str:
    value = executor_id.value if hasattr(executor_id, "value") else executor_id
    return _extract(value, False)


def to_sanitized_service_name_from_id(any_id) -> Optional[str]:
    value = any_id.value if hasattr(any_id, "value") else any_id
    return _extract(value, True)


def empty_task_id() -> P.TaskID:
    return P.TaskID(value="")


def empty_agent_id() -> P.AgentID:
    return P.AgentID(value="")


def get_task_instance_name(pod_instance, task) -> str:
    name = task if isinstance(task, str) else task.name
    return f"{pod_instance.name}-{name}"
