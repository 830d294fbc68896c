"""Builds the ``TaskInfo``/``ExecutorInfo`` protos for one pod instance.

Reference: sdk/.../offer/evaluate/PodInfoBuilder.java:72-831. Stages mutate the builders held
here; ``LaunchEvaluationStage`` snapshots them into launch / store recommendations.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Set

from dcos_commons_amd.http import endpoint_utils as eu
from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.offer import common_id_utils
from dcos_commons_amd.offer import constants
from dcos_commons_amd.offer.evaluate import placement
from dcos_commons_amd.offer.resources import ResourceBuilder
from dcos_commons_amd.offer.taskdata import labels as L
from dcos_commons_amd.specification.specs import (
    RLIMIT_INFINITY,
    ConfigFileSpec,
    PodInstance,
    PodSpec,
    ReadinessCheckSpec,
    TaskSpec,
    VolumeSpec,
)
from dcos_commons_amd.state.goal_state_override import PAUSE_READINESS_COMMAND, GoalStateOverride

CONFIG_TEMPLATE_KEY_FORMAT = "CONFIG_TEMPLATE_%s"
CONFIG_TEMPLATE_DOWNLOAD_PATH = "config-templates/"


class InvalidRequirementException(Exception):
    pass


def get_task_environment(service_name: str, pod_instance: PodInstance, task_spec: TaskSpec,
                         scheduler_config) -> Dict[str, str]:
    env: Dict[str, str] = {}
    if task_spec.command is not None:
        env.update(task_spec.command.env)
    env.update(_instance_environment(service_name, pod_instance, task_spec, scheduler_config))
    return dict(sorted(env.items()))


def _instance_environment(service_name: str, pod_instance: PodInstance, task_spec: TaskSpec,
                          scheduler_config) -> Dict[str, str]:
    """The variables every task gets on top of its spec's ``env`` (PodInfoBuilder.getTaskEnvironment)."""
    env: Dict[str, str] = {}
    task_name = f"{pod_instance.name}-{task_spec.name}"
    env[L.POD_INSTANCE_INDEX_TASKENV] = str(pod_instance.index)
    env[L.FRAMEWORK_NAME_TASKENV] = service_name
    env[L.FRAMEWORK_HOST_TASKENV] = eu.to_auto_ip_domain(service_name, scheduler_config)
    env[L.FRAMEWORK_VIP_HOST_TASKENV] = eu.to_vip_domain(service_name, scheduler_config)
    env[L.SCHEDULER_API_HOSTNAME_TASKENV] = eu.to_scheduler_auto_ip_hostname(service_name, scheduler_config)
    env[L.SCHEDULER_API_PORT_TASKENV] = str(scheduler_config.api_server_port())
    env[L.TASK_NAME_TASKENV] = task_name
    env[task_name] = "true"
    env[L.PLACEMENT_REFERENCED_REGION_ENV] = str(placement.references_region(pod_instance.pod)).lower()
    env[L.PLACEMENT_REFERENCED_ZONE_ENV] = str(placement.references_zone(pod_instance.pod)).lower()
    return env


def _environment_bytes(service_name: str, pod_instance: PodInstance, task_spec: TaskSpec, scheduler_config,
                       more: Optional[Dict[str, str]] = None) -> bytes:
    """``get_task_environment`` (plus ``more``) as a serialized, name-sorted ``Environment``, from
    the spec env's cached pre-encoded template and the per-instance variables."""
    extra = _instance_environment(service_name, pod_instance, task_spec, scheduler_config)
    if more:
        extra.update(more)
    static = task_spec.command.environment if task_spec.command is not None else ()
    return L.env_template(static).encode(extra)


def _move_environment(env: P.Environment, old_name: str, new_name: str, index: str, tail: int = 0) -> bool:
    """Rewrites the per-instance variables of a task environment in place (see
    ``PodInfoBuilder.for_instance``); False when the result would not be what a fresh build
    gives."""
    vs = env.variables
    slot = -1
    fixed = 0
    for i, v in enumerate(vs):
        name = v.name
        if name == old_name:
            if slot >= 0:
                return False
            slot = i
        elif name == new_name:
            return False
        elif name == L.POD_INSTANCE_INDEX_TASKENV:
            v.value = index
            fixed += 1
        elif name == L.TASK_NAME_TASKENV:
            v.value = new_name
            fixed += 1
    if slot < 0 or fixed != 2:
        return False
    # the task-name variable keeps its slot only if the new name sorts there too, among the
    # name-sorted variables (the last ``tail`` ones were appended after them)
    end = len(vs) - tail
    if slot >= end:
        return False
    if slot > 0 and not vs[slot - 1].name < new_name:
        return False
    if slot + 1 < end and not new_name < vs[slot + 1].name:
        return False
    vs[slot].name = new_name
    return True


def config_template_download_path(config: ConfigFileSpec) -> str:
    return CONFIG_TEMPLATE_DOWNLOAD_PATH + config.name


def _reference_secret(path: str) -> P.Secret:
    s = P.Secret(type=P.Secret.REFERENCE)
    s.reference.name = path
    return s


class PodInfoBuilder:
    def __init__(self, requirement, service_name: str, target_config_id, template_url_factory, scheduler_config,
                 current_pod_tasks, framework_id: P.FrameworkID, override_map: Dict[str, GoalStateOverride]):
        pi: PodInstance = requirement.pod_instance
        self.pod_instance = pi
        # variables appended after a command environment's name-sorted part: the requirement's
        # environment, then the pod's environment secrets (for_instance)
        self._env_tail = len(requirement.environment) + sum(1 for x in pi.pod.secrets if x.env_key is not None)
        self.assigned_overlay_ports: Set[int] = set()
        self.task_builders: Dict[str, P.TaskInfo] = {}
        for ts in pi.pod.tasks:
            self.task_builders[ts.name] = self._create_task_info(
                pi, ts, requirement.environment, service_name, target_config_id, template_url_factory,
                scheduler_config, override_map.get(ts.name, GoalStateOverride.NONE))
            for rs in ts.resource_set.resources:
                if rs.name == constants.PORTS_RESOURCE_TYPE and rs.value.ranges.range[0].begin > 0:
                    self.assigned_overlay_ports.add(int(rs.value.ranges.range[0].begin))
        self.executor_builder = self._executor_info(pi, framework_id, scheduler_config)
        self.ports_by_task: Dict[str, Dict[str, int]] = self.prior_ports(current_pod_tasks)
        for tb in self.task_builders.values():
            self._validate(tb)

    @staticmethod
    def prior_ports(current_pod_tasks) -> Dict[str, Dict[str, int]]:
        """Ports the pod's current (not permanently failed) tasks hold, by task and port name: a
        relaunch keeps them. Read-only once built; builders of one evaluation share it."""
        out: Dict[str, Dict[str, int]] = {}
        for t in current_pod_tasks:
            if not L.TaskLabelReader(t).is_permanently_failed():
                out[t.name] = {p.name: int(p.number) for p in t.discovery.ports.ports if p.name}
        return out

    def clone(self) -> "PodInfoBuilder":
        """A builder in the state this one was constructed in, for the next offer. Nothing in the
        construction but ``ports_by_task`` depends on the offer or the pod's current tasks, so the
        evaluator keeps one untouched template per (pod instance, target config, requirement
        environment, goal overrides) across offer cycles, and each offer's stages mutate a copy
        (protobuf ``CopyFrom``) instead of rebuilding every task's command, environment, checks and
        container info (a reference hdfs/cassandra task carries hundreds of environment variables).
        Call it on a builder no stage has touched."""
        c = PodInfoBuilder.__new__(PodInfoBuilder)
        c.pod_instance = self.pod_instance
        c._env_tail = self._env_tail
        c.assigned_overlay_ports = set(self.assigned_overlay_ports)
        c.task_builders = {}
        for name, tb in self.task_builders.items():
            t = P.TaskInfo()
            t.CopyFrom(tb)
            c.task_builders[name] = t
        c.executor_builder = P.ExecutorInfo()
        c.executor_builder.CopyFrom(self.executor_builder)
        c.ports_by_task = self.ports_by_task  # read-only after construction
        return c

    def for_instance(self, pi: PodInstance) -> Optional["PodInfoBuilder"]:
        """This untouched template moved to another instance of the same pod (same requirement
        environment, target config and goal overrides), or None where that cannot be done exactly.

        A fresh builder for instance ``pi`` differs from this one's copy only in what the pod
        index reaches: each task's name, its ``index`` label, its discovery name, and in the task
        environments (command, health check, readiness check) the ``POD_INSTANCE_INDEX`` and
        ``TASK_NAME`` values and the variable named after the task. That variable sits in the
        name-sorted part of the environment; when the new name does not sort into the old slot,
        or a name is ambiguous, the caller builds from scratch. A parallel deploy of N instances
        builds the pod's task templates once instead of N times."""
        old = self.pod_instance
        if pi.pod is not old.pod:
            return None
        c = self.clone()
        c.pod_instance = pi
        index = str(pi.index)
        for ts in pi.pod.tasks:
            t = c.task_builders.get(ts.name)
            if t is None:
                return None
            old_name, new_name = f"{old.name}-{ts.name}", f"{pi.name}-{ts.name}"
            if t.name != old_name:
                return None
            t.name = new_name
            found = 0
            for label in t.labels.labels:
                if label.key == L.TASK_INDEX_LABEL:
                    label.value = index
                    found += 1
            if found != 1:
                return None
            if ts.discovery is not None and ts.discovery.prefix:
                t.discovery.name = f"{ts.discovery.prefix}-{pi.index}"
            envs = []
            if t.HasField("command"):
                envs.append((t.command.environment, self._env_tail))
            if t.HasField("health_check"):
                envs.append((t.health_check.command.environment, 0))
            if t.HasField("check"):
                envs.append((t.check.command.command.environment, 0))
            for env, tail in envs:
                if not _move_environment(env, old_name, new_name, index, tail):
                    return None
        return c

    # -- accessors ---------------------------------------------------------------------
    def get_task_builders(self) -> List[P.TaskInfo]:
        return list(self.task_builders.values())

    def get_task_builder(self, task_spec_name: str) -> P.TaskInfo:
        return self.task_builders[task_spec_name]

    def get_executor_builder(self) -> Optional[P.ExecutorInfo]:
        return self.executor_builder

    def get_prior_port_for_task(self, task_spec_name: str, port_spec) -> Optional[int]:
        ports = self.ports_by_task.get(f"{self.pod_instance.name}-{task_spec_name}")
        if ports is None:
            return None
        return ports.get(port_spec.port_name)

    def get_task_resources(self) -> List[P.Resource]:
        return [r for t in self.task_builders.values() for r in t.resources]

    def get_executor_resources(self) -> List[P.Resource]:
        return list(self.executor_builder.resources)

    def is_assigned_overlay_port(self, port: int) -> bool:
        return port in self.assigned_overlay_ports

    def add_assigned_overlay_port(self, port: int) -> None:
        self.assigned_overlay_ports.add(port)

    @property
    def type(self) -> str:
        return self.pod_instance.pod.type

    @property
    def index(self) -> int:
        return self.pod_instance.index

    def set_executor_volume(self, volume_spec: VolumeSpec) -> None:
        vol = P.Volume(mode=P.Volume.RW, container_path=volume_spec.container_path)
        vol.source.type = P.Volume.Source.SANDBOX_PATH
        vol.source.sandbox_path.type = P.Volume.Source.SandboxPath.PARENT
        vol.source.sandbox_path.path = volume_spec.container_path
        for t in self.task_builders.values():
            t.container.type = P.ContainerInfo.MESOS
            t.container.volumes.add().CopyFrom(vol)

    @staticmethod
    def get_existing_executor_volume(volume_spec, resource_id, resource_namespace, persistence_id, provider_id,
                                     disk_source, framework_id) -> P.Resource:
        return ResourceBuilder.from_volume_spec(volume_spec, resource_id, resource_namespace, persistence_id,
                                                provider_id, disk_source, framework_id).build()

    # -- construction ------------------------------------------------------------------
    def _create_task_info(self, pi: PodInstance, ts: TaskSpec, environment: Dict[str, str], service_name: str,
                          target_config_id, template_url_factory, scheduler_config,
                          override: GoalStateOverride) -> P.TaskInfo:
        pod = pi.pod
        t = P.TaskInfo(name=f"{pi.name}-{ts.name}")
        t.task_id.value = ""
        t.agent_id.value = ""
        w = L.TaskLabelWriter(t).set_target_configuration(target_config_id).set_type(pod.type).set_index(pi.index)
        w.set_additional_labels(ts.labels)
        w.apply()
        # the command, health check and readiness check all start from the same task environment
        base_env = P.Environment()
        base_env.MergeFromString(_environment_bytes(service_name, pi, ts, scheduler_config))
        if ts.command is not None:
            cmd = t.command
            if ts.config_files:
                # EnvUtils.withEnvVar per config file (PodInfoBuilder.java:279-283): keyed by name,
                # sorted; merged in one pass rather than re-sorting the proto per file
                more = {CONFIG_TEMPLATE_KEY_FORMAT % L.to_env_name(config.name):
                        f"{config_template_download_path(config)},{config.relative_path}" for config in ts.config_files}
                cmd.environment.MergeFromString(_environment_bytes(service_name, pi, ts, scheduler_config, more))
            else:
                cmd.environment.CopyFrom(base_env)
            if override == GoalStateOverride.PAUSED:
                cmd.value = scheduler_config.pause_override_cmd()
            else:
                cmd.value = ts.command.value
            for k, v in environment.items():
                cmd.environment.variables.add(name=k, value=v)
            if override == GoalStateOverride.PAUSED:
                cmd.uris.add(value=scheduler_config.bootstrap_uri())
            for uri in pod.uris:
                cmd.uris.add(value=uri)
            for config in ts.config_files:
                cmd.uris.add(value=template_url_factory(target_config_id, pod.type, ts.name, config.name),
                             output_file=config_template_download_path(config), extract=False)
            for secret in pod.secrets:
                if secret.env_key is not None:
                    v = cmd.environment.variables.add(name=secret.env_key, type=P.Environment.Variable.SECRET)
                    v.secret.CopyFrom(_reference_secret(secret.secret_path))
            if pod.user:
                cmd.user = pod.user
        if ts.discovery is not None:
            d = t.discovery
            if ts.discovery.prefix:
                d.name = f"{ts.discovery.prefix}-{pi.index}"
            d.visibility = (ts.discovery.visibility if ts.discovery.visibility is not None
                            else constants.DEFAULT_TASK_DISCOVERY_VISIBILITY)
        t.container.CopyFrom(self._container_info(pod, True, True))
        if ts.shared_memory is not None:
            t.container.linux_info.ipc_mode = P.LinuxInfo.IpcMode.Value(ts.shared_memory.value)
        if ts.shared_memory_size is not None:
            t.container.linux_info.shm_size = ts.shared_memory_size
        self._set_health_check(t, service_name, pi, ts, override, scheduler_config, base_env)
        self._set_readiness_check(t, service_name, pi, ts, override, scheduler_config, base_env)
        if ts.kill_grace_period < 0:
            raise InvalidRequirementException(
                f"kill-grace-period must be zero or a positive integer, received: {ts.kill_grace_period}")
        t.kill_policy.grace_period.nanoseconds = 1_000_000_000 * int(ts.kill_grace_period or 0)
        return t

    @staticmethod
    def _set_health_check(t, service_name, pi, ts, override, scheduler_config, env=None) -> None:
        hc = ts.health_check
        if hc is None or override == GoalStateOverride.PAUSED:
            return
        h = t.health_check
        h.delay_seconds = hc.delay
        h.interval_seconds = hc.interval
        h.timeout_seconds = hc.timeout
        h.consecutive_failures = hc.max_consecutive_failures
        h.grace_period_seconds = hc.grace_period
        h.type = P.HealthCheck.COMMAND
        h.command.value = hc.command
        h.command.environment.CopyFrom(
            env if env is not None else L.env_from_map(get_task_environment(service_name, pi, ts, scheduler_config)))

    @staticmethod
    def _set_readiness_check(t, service_name, pi, ts, override, scheduler_config, env=None) -> None:
        rc = ts.readiness_check
        if override == GoalStateOverride.PAUSED:
            rc = ReadinessCheckSpec(PAUSE_READINESS_COMMAND, constants.SHORT_DECLINE_SECONDS,
                                    constants.SHORT_DECLINE_SECONDS)
        if rc is None:
            return
        c = t.check
        c.type = P.CheckInfo.COMMAND
        c.delay_seconds = rc.delay
        c.interval_seconds = rc.interval
        c.timeout_seconds = rc.timeout
        c.command.command.value = rc.command
        c.command.command.environment.CopyFrom(
            env if env is not None else L.env_from_map(get_task_environment(service_name, pi, ts, scheduler_config)))

    @staticmethod
    def _executor_info(pi: PodInstance, framework_id: P.FrameworkID, scheduler_config) -> P.ExecutorInfo:
        e = P.ExecutorInfo(name=pi.pod.type)
        e.executor_id.value = ""
        L.set_dcos_space(e, scheduler_config.dcos_space())
        e.type = P.ExecutorInfo.DEFAULT
        e.framework_id.CopyFrom(framework_id)
        e.container.CopyFrom(PodInfoBuilder._container_info(pi.pod, True, False))
        return e

    @staticmethod
    def _container_info(pod: PodSpec, add_extra: bool, is_task: bool) -> P.ContainerInfo:
        c = P.ContainerInfo(type=P.ContainerInfo.MESOS)
        secret_vols = []
        for s in pod.secrets:
            if s.file_path is not None:
                v = P.Volume(container_path=s.file_path, mode=P.Volume.RO)
                v.source.type = P.Volume.Source.SECRET
                v.source.secret.CopyFrom(_reference_secret(s.secret_path))
                secret_vols.append(v)
        if is_task:
            c.linux_info.share_pid_namespace = bool(pod.share_pid_namespace)
            c.volumes.add(container_path="/tmp", host_path="tmp", mode=P.Volume.RW)
            if pod.seccomp_unconfined:
                c.linux_info.seccomp.unconfined = True
            if pod.seccomp_profile_name:
                c.linux_info.seccomp.Clear()
                c.linux_info.seccomp.profile_name = pod.seccomp_profile_name
        else:
            if pod.shared_memory is not None:
                c.linux_info.ipc_mode = P.LinuxInfo.IpcMode.Value(pod.shared_memory.value)
            if pod.shared_memory_size is not None:
                c.linux_info.shm_size = pod.shared_memory_size
        for hv in pod.host_volumes:
            c.volumes.add(host_path=hv.host_path, container_path=hv.container_path,
                          mode=P.Volume.Mode.Value(hv.mode) if hv.mode else P.Volume.RW)
        if not pod.image and not pod.networks and not pod.rlimits and not secret_vols:
            return c
        if pod.image and add_extra and is_task:
            c.mesos.image.type = P.Image.DOCKER
            c.mesos.image.docker.name = pod.image
        if pod.networks and not is_task:
            for n in pod.networks:
                ni = c.network_infos.add(name=n.name)
                for hp, cp in n.port_mappings:
                    ni.port_mappings.add(host_port=hp, container_port=cp)
                if n.labels:
                    L.map_to_labels(dict(n.labels), ni.labels)
        if pod.rlimits and add_extra:
            for rl in pod.rlimits:
                r = c.rlimit_info.rlimits.add(type=rl.enum)
                if rl.soft is not None and rl.hard is not None and rl.soft != RLIMIT_INFINITY and \
                        rl.hard != RLIMIT_INFINITY:
                    r.soft = rl.soft
                    r.hard = rl.hard
        if add_extra:
            for v in secret_vols:
                c.volumes.add().CopyFrom(v)
        return c

    @staticmethod
    def _validate(t: P.TaskInfo) -> None:
        if not t.name:
            raise InvalidRequirementException(f"TaskInfo must have a name: {t}")
        if t.task_id.value:
            try:
                name = common_id_utils.to_task_name(t.task_id)
            except L.TaskException as e:
                raise InvalidRequirementException(f"When non-empty, TaskInfo.id must be a valid ID: {e}")
            if name != t.name:
                raise InvalidRequirementException("When non-empty, TaskInfo.id must align with TaskInfo.name")
        if t.HasField("executor"):
            raise InvalidRequirementException("TaskInfo must not contain ExecutorInfo.")
        reader = L.TaskLabelReader(t)
        try:
            reader.get_type()
            reader.get_index()
        except (L.TaskException, ValueError) as e:
            raise InvalidRequirementException(str(e))
