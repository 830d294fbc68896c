"""TaskUtils and CommonIdUtils.

Mirrors the reference's offer/{TaskUtilsTest,CommonIdUtilsTest}.java (sdk/scheduler/src/test/java/
com/mesosphere/sdk/offer/): ID construction and parsing (foldered service names, extra leading
elements, underscores next to the delimiter, malformed IDs), spec diffing that decides whether a
task must be relaunched, which stored tasks need recovery, and how failed tasks are grouped into
per-pod recovery requirements (an essential task failing relaunches its whole pod, non-essential
ones relaunch alone; launch backoff holds them back; ONCE tasks are never recovered).
"""
import uuid

import pytest

from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.offer import common_id_utils as C
from dcos_commons_amd.offer import task_utils as T
from dcos_commons_amd.offer.taskdata.labels import TaskException, TaskLabelWriter
from dcos_commons_amd.scheduler.plan import backoff as B
from dcos_commons_amd.scheduler.scheduler_config import SchedulerConfig
from dcos_commons_amd.specification.specs import loopback_check
from dcos_commons_amd.specification.yaml import mappers
from dcos_commons_amd.specification.yaml.raw import RawServiceSpec
from dcos_commons_amd.state.config_store import ConfigStore
from dcos_commons_amd.storage.mem_persister import MemPersister

SVC = "test-service_name"
FOLDERED = "/path/to/test-service_name"
FOLDERED2 = "path/to.test-service_name"
SANITIZED = "path.to.test-service_name"
TASK = "test_task-name"
OTHER = "test-other_name"


# ---------------------------------------------------------------------------------------
# CommonIdUtils


@pytest.mark.parametrize("name,expected", [
    ("/path/to/service", "path.to.service"), ("//path/to/service///", "path.to.service"),
    ("path/to/service", "path.to.service"), ("/service", "service"), ("///service//", "service"),
])
def test_sanitized_service_names(name, expected):
    assert C.to_sanitized_service_name(name) == expected


@pytest.mark.parametrize("kind", ["task", "executor"])
@pytest.mark.parametrize("value,name,service", [
    (TASK + "__id", TASK, None),
    ("___id", "_", None),
    (OTHER + "__" + TASK + "__id", TASK, OTHER),
    (OTHER + "___" + TASK + "__id", TASK, OTHER + "_"),
    ("_" + OTHER + "___" + TASK + "__id", TASK, "_" + OTHER + "_"),
    (OTHER + "____id", "", OTHER),
    (OTHER + "___id", OTHER + "_", None),
    ("_" + OTHER + "___id", "_" + OTHER + "_", None),
    # extra leading elements are tolerated (reserved for future use)
    ("something-else__" + FOLDERED2 + "__" + TASK + "__uuid", TASK, FOLDERED2),
])
def test_name_and_service_extraction(kind, value, name, service):
    i = P.TaskID(value=value) if kind == "task" else P.ExecutorID(value=value)
    to_name = C.to_task_name if kind == "task" else C.to_executor_name
    assert to_name(i) == name
    assert C.to_sanitized_service_name_from_id(i) == service


@pytest.mark.parametrize("kind", ["task", "executor"])
@pytest.mark.parametrize("service,sanitized", [(SVC, SVC), (FOLDERED, SANITIZED), (FOLDERED2, SANITIZED)])
def test_id_construction_round_trip(kind, service, sanitized):
    make = C.to_task_id if kind == "task" else C.to_executor_id
    to_name = C.to_task_name if kind == "task" else C.to_executor_name
    i = make(service, TASK)
    assert i.value.startswith(f"{sanitized}__{TASK}__")
    uuid.UUID(i.value.split("__")[2])
    assert to_name(i) == TASK
    assert C.to_sanitized_service_name_from_id(i) == sanitized
    assert make(service, TASK).value != i.value  # a fresh UUID every time


@pytest.mark.parametrize("make", [C.to_task_id, C.to_executor_id])
def test_double_underscores_are_reserved(make):
    with pytest.raises(ValueError):
        make(OTHER + "__" + SVC, TASK)
    with pytest.raises(ValueError):
        make(SVC, OTHER + "__" + TASK)


@pytest.mark.parametrize("to_name,make", [(C.to_task_name, P.TaskID), (C.to_executor_name, P.ExecutorID)])
def test_malformed_ids(to_name, make):
    with pytest.raises(TaskException):
        to_name(make(value=TASK + "_id"))


def test_task_instance_name():
    class PI:
        name = "pod-3"
    assert C.get_task_instance_name(PI(), "server") == "pod-3-server"


# ---------------------------------------------------------------------------------------
# are_different


BASE = """\
name: svc
pods:
  pod:
    count: 1
    {rs}
    tasks:
      {name}:
        goal: {goal}
        cmd: "{cmd}"
        {res}
        {configs}
"""


def _task_spec(tmp_path, name="task", goal="RUNNING", cmd="echo hi", res="cpus: 1\n        memory: 2",
               configs="", resource_set=None, templates=None):
    for fname, content in (templates or {}).items():
        (tmp_path / fname).write_text(content)
    rs = ""
    if resource_set is not None:
        rs = "resource-sets:\n      " + resource_set[0] + ":\n" + "".join(
            f"        {k}: {v}\n" for k, v in resource_set[1].items())
        res = f"resource-set: {resource_set[0]}"
    raw = RawServiceSpec.from_string(BASE.format(name=name, goal=goal, cmd=cmd, res=res, configs=configs, rs=rs))
    spec = mappers.ServiceSpecGenerator(raw, SchedulerConfig.for_testing(), str(tmp_path), {}).build()
    return spec.pods[0].tasks[0]


def test_identical_specs_are_not_different(tmp_path):
    assert not T.are_different(_task_spec(tmp_path), _task_spec(tmp_path))


@pytest.mark.parametrize("change", [dict(name="newtask"), dict(cmd="echo hi && echo foo"), dict(goal="ONCE"),
                                    dict(res="cpus: 1\n        memory: 2\n        gpus: 1"),
                                    dict(res="cpus: 1"), dict(res="memory: 2\n        cpus: 5")])
def test_relevant_changes_make_specs_different(tmp_path, change):
    assert T.are_different(_task_spec(tmp_path), _task_spec(tmp_path, **change))


def test_resource_set_id_alone_does_not_matter(tmp_path):
    a = _task_spec(tmp_path, resource_set=("rs-a", {"cpus": 5, "memory": 3}))
    b = _task_spec(tmp_path, resource_set=("rs-b", {"cpus": 5, "memory": 3}))
    assert not T.are_different(a, b)
    c = _task_spec(tmp_path, resource_set=("rs-a", {"cpus": 5}))
    d = _task_spec(tmp_path, resource_set=("rs-a", {"memory": 5}))
    assert T.are_different(c, d)  # no overlap at all


CONFIGS = ("configs:\n          config:\n            template: c1.tmpl\n            dest: ../relative/path/to/config\n"
           "          config2:\n            template: c2.tmpl\n            dest: ../relative/path/to/config2")
CONFIGS_REORDERED = ("configs:\n          config2:\n            template: c2.tmpl\n"
                     "            dest: ../relative/path/to/config2\n          config:\n"
                     "            template: c1.tmpl\n            dest: ../relative/path/to/config")


def test_config_templates_are_compared_by_content_not_order(tmp_path):
    base = dict(configs=CONFIGS, templates={"c1.tmpl": "a config template", "c2.tmpl": "second config"})
    a = _task_spec(tmp_path, **base)
    b = _task_spec(tmp_path, configs=CONFIGS_REORDERED, templates={"c1.tmpl": "a config template",
                                                                    "c2.tmpl": "second config"})
    assert not T.are_different(a, b)
    c = _task_spec(tmp_path, configs=CONFIGS, templates={"c1.tmpl": "a diff config template",
                                                         "c2.tmpl": "diff second config"})
    assert T.are_different(a, c)
    assert T.are_different(_task_spec(tmp_path), a)  # configs added


# ---------------------------------------------------------------------------------------
# recovery selection and pod requirements


LAYOUT = """\
name: svc
pods:
  server:
    count: 3
    tasks:
{tasks}
      once:
        goal: ONCE
        cmd: echo once
        cpus: 0.1
        memory: 32
"""


def _layout(essential: int, nonessential: int):
    tasks = ""
    for i in range(essential):
        tasks += f"      essential{i}:\n        goal: RUNNING\n        cmd: echo e{i}\n        cpus: 0.1\n        memory: 32\n"
    for i in range(nonessential):
        tasks += (f"      nonessential{i}:\n        goal: RUNNING\n        essential: false\n        cmd: echo n{i}\n"
                  f"        cpus: 0.1\n        memory: 32\n")
    raw = RawServiceSpec.from_string(LAYOUT.format(tasks=tasks))
    spec = mappers.ServiceSpecGenerator(raw, SchedulerConfig.for_testing(), "/tmp", {}).build()
    cs = ConfigStore(loopback_check(spec), MemPersister())
    target = cs.store(spec)
    cs.set_target_config(target)
    infos = []
    for idx in range(3):
        for t in spec.pods[0].tasks:
            if t.name == "once":
                continue
            infos.append(_info(f"server-{idx}-{t.name}", "server", idx, target))
    return cs, infos


def _info(name, pod_type, index, target):
    t = P.TaskInfo(name=name)
    t.task_id.CopyFrom(C.to_task_id("svc", name))
    t.agent_id.value = "agent"
    w = TaskLabelWriter(t)
    w.set_type(pod_type)
    w.set_index(index)
    w.set_target_configuration(target)
    w.apply()
    return t


def _staging(infos):
    return [P.TaskStatus(task_id=t.task_id, state=P.TASK_STAGING) for t in infos]


def _pick(infos, *names):
    return [t for t in infos if t.name in names]


class FixedBackoff:
    def __init__(self, delayed=()):
        self.delayed = set(delayed)

    def get_delay(self, name):
        return 1.0 if name in self.delayed else None


def _reqs(layout, failed, backoff=None):
    cs, infos = layout
    return T.get_pod_requirements(cs, infos, _staging(infos), _pick(infos, *failed), backoff or FixedBackoff())


ALL4 = ["essential0", "essential1", "nonessential0", "nonessential1"]


@pytest.fixture(scope="module")
def mixed():
    return _layout(2, 2)


def test_failed_essential_tasks_relaunch_their_whole_pods(mixed):
    reqs = _reqs(mixed, ["server-0-essential0", "server-0-essential1", "server-1-essential1"])
    assert [(r.name, list(r.tasks_to_launch)) for r in reqs] == [
        ("server-0:[essential0, essential1, nonessential0, nonessential1]", ALL4),
        ("server-1:[essential0, essential1, nonessential0, nonessential1]", ALL4)]


def test_failed_non_essential_tasks_relaunch_alone(mixed):
    reqs = _reqs(mixed, ["server-0-nonessential0", "server-0-nonessential1", "server-1-nonessential1"])
    assert [(r.name, list(r.tasks_to_launch)) for r in reqs] == [
        ("server-0:[nonessential0, nonessential1]", ["nonessential0", "nonessential1"]),
        ("server-1:[nonessential1]", ["nonessential1"])]


def test_mixed_failures(mixed):
    reqs = _reqs(mixed, ["server-0-essential0", "server-0-nonessential0", "server-1-nonessential1"])
    assert [r.name for r in reqs] == ["server-0:[essential0, essential1, nonessential0, nonessential1]",
                                      "server-1:[nonessential1]"]


def test_all_essential_and_all_non_essential_pods():
    reqs = _reqs(_layout(2, 0), ["server-0-essential0", "server-0-essential1", "server-1-essential1"])
    assert [r.name for r in reqs] == ["server-0:[essential0, essential1]", "server-1:[essential0, essential1]"]
    reqs = _reqs(_layout(0, 2), ["server-0-nonessential0", "server-0-nonessential1", "server-1-nonessential1"])
    assert [r.name for r in reqs] == ["server-0:[nonessential0, nonessential1]", "server-1:[nonessential1]"]


def test_delayed_essential_task_holds_back_its_pod(mixed):
    failed = ["server-0-essential0", "server-1-essential0", "server-0-nonessential0", "server-1-nonessential0",
              "server-2-nonessential0", "server-0-nonessential1", "server-1-nonessential1",
              "server-2-nonessential1"]
    reqs = _reqs(mixed, failed, FixedBackoff(["server-0-essential0", "server-1-essential0"]))
    assert [r.name for r in reqs] == ["server-2:[nonessential0, nonessential1]"]


def test_delayed_non_essential_task_holds_back_an_essential_relaunch_of_its_pod(mixed):
    failed = ["server-0-essential0", "server-1-essential0", "server-2-nonessential0", "server-2-nonessential1"]
    reqs = _reqs(mixed, failed, FixedBackoff(["server-0-nonessential0", "server-1-nonessential0"]))
    assert [r.name for r in reqs] == ["server-2:[nonessential0, nonessential1]"]


def test_delayed_non_essential_tasks_are_skipped_individually():
    layout = _layout(0, 2)
    failed = [f"server-{i}-nonessential{j}" for j in (0, 1) for i in range(3)]
    delayed = ["server-0-nonessential0", "server-0-nonessential1", "server-1-nonessential0", "server-2-nonessential1"]
    reqs = _reqs(layout, failed, FixedBackoff(delayed))
    assert [r.name for r in reqs] == ["server-1:[nonessential1]", "server-2:[nonessential0]"]


def test_tasks_never_launched_are_not_relaunched(mixed):
    cs, infos = mixed
    statuses = _staging([t for t in infos if t.name != "server-0-essential1"])
    reqs = T.get_pod_requirements(cs, infos, statuses, _pick(infos, "server-0-essential0"), FixedBackoff())
    assert [r.name for r in reqs] == ["server-0:[essential0, nonessential0, nonessential1]"]


def test_recovery_needed_states():
    lost = P.TaskStatus(state=P.TASK_LOST)
    lost.task_id.value = str(uuid.uuid4())
    assert T.is_recovery_needed(lost)
    # terminal states (FINISHED too: recovery only applies to RUNNING-goal tasks) plus LOST/UNREACHABLE
    for st in (P.TASK_FAILED, P.TASK_KILLED, P.TASK_ERROR, P.TASK_FINISHED, P.TASK_DROPPED, P.TASK_GONE,
               P.TASK_LOST, P.TASK_UNREACHABLE):
        assert T.is_recovery_needed(P.TaskStatus(state=st)), P.TaskState.Name(st)
    # GONE_BY_OPERATOR goes through replacement instead (get_tasks_for_replacement)
    for st in (P.TASK_STAGING, P.TASK_STARTING, P.TASK_RUNNING, P.TASK_KILLING, P.TASK_GONE_BY_OPERATOR,
               P.TASK_UNKNOWN):
        assert not T.is_recovery_needed(P.TaskStatus(state=st)), P.TaskState.Name(st)


SEQ = """\
name: svc
pods:
  name:
    count: 1
    tasks:
      format:
        goal: ONCE
        cmd: ./format
        cpus: 0.1
        memory: 32
      node:
        goal: RUNNING
        cmd: ./node
        cpus: 0.1
        memory: 32
"""


@pytest.fixture
def seq():
    raw = RawServiceSpec.from_string(SEQ)
    spec = mappers.ServiceSpecGenerator(raw, SchedulerConfig.for_testing(), "/tmp", {}).build()
    cs = ConfigStore(loopback_check(spec), MemPersister())
    target = cs.store(spec)
    cs.set_target_config(target)
    return cs, target


def _st(info, state):
    return P.TaskStatus(task_id=info.task_id, state=state)


def test_no_tasks_or_no_statuses_need_no_recovery(seq):
    cs, target = seq
    assert T.get_tasks_needing_recovery(None, [], []) == []
    t = _info("name-0-node", "name", 0, target)
    assert T.get_tasks_needing_recovery(cs, [t], []) == []


@pytest.mark.parametrize("task,state,needed", [
    ("node", P.TASK_RUNNING, False), ("node", P.TASK_FAILED, True),
    ("format", P.TASK_FAILED, False), ("format", P.TASK_FINISHED, False), ("format", P.TASK_RUNNING, False),
])
def test_tasks_needing_recovery_by_goal_and_state(seq, task, state, needed):
    cs, target = seq
    t = _info(f"name-0-{task}", "name", 0, target)
    assert T.get_tasks_needing_recovery(cs, [t], [_st(t, state)]) == ([t] if needed else [])


def test_unknown_task_in_the_spec_raises(seq):
    cs, target = seq
    t = _info("name-0-not-present", "name", 0, target)
    with pytest.raises(TaskException):
        T.get_tasks_needing_recovery(cs, [t], [_st(t, P.TASK_RUNNING)])
    assert T.get_tasks_needing_recovery(cs, [t], []) == []  # without a status it is never looked up


def test_permanently_failed_running_task_needs_recovery(seq):
    cs, target = seq
    t = _info("name-0-node", "name", 0, target)
    running = _st(t, P.TASK_RUNNING)
    TaskLabelWriter(t).set_permanently_failed().apply()
    assert T.get_tasks_needing_recovery(cs, [t], [running]) == [t]


def test_gone_by_operator_tasks_are_replaced_once(seq):
    _, target = seq
    t = _info("name-0-node", "name", 0, target)
    gone = _st(t, P.TASK_GONE_BY_OPERATOR)
    assert T.get_tasks_for_replacement([gone], [t]) == [t]
    TaskLabelWriter(t).set_permanently_failed().apply()
    assert T.get_tasks_for_replacement([gone], [t]) == []  # already marked
    assert T.get_tasks_for_replacement([_st(t, P.TASK_LOST)], [t]) == []


def test_pod_instance_resolution_uses_the_launch_config(seq):
    cs, target = seq
    t = _info("name-0-node", "name", 0, target)
    pi = T.get_pod_instance(cs, t)
    assert pi.name == "name-0" and T.get_task_spec(pi, t.name).name == "node"
    bad = _info("name-0-node", "name", 0, uuid.uuid4())
    with pytest.raises(TaskException):
        T.get_pod_instance(cs, bad)
    nopod = _info("other-0-node", "other", 0, target)
    with pytest.raises(TaskException):
        T.get_pod_instance(cs, nopod)


@pytest.fixture(autouse=True)
def _no_global_backoff():
    B.set_instance(B.DisabledBackoff())
    yield
    B.set_instance(None)
