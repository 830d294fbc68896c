"""Registers a framework with Mesos and runs it.

Reference: sdk/.../framework/FrameworkRunner.java:60-230. Builds the FrameworkInfo (2-week
failover timeout, checkpointing, MULTI_ROLE when >1 role, PARTITION_AWARE, GPU_RESOURCES when
any pod asks for GPUs, RESERVATION_REFINEMENT, REGION_AWARE), starts the API server (offers are
declined until it is up), creates the driver and blocks on it. With uninstall enabled and no
stored FrameworkID it wipes the state and serves an empty deploy plan ("skeleton scheduler").

Drivers: ``driver_factory(scheduler, framework_info) -> driver``. The default
(``scheduler_driver_factory``) picks from ``SDK_MESOS_MASTER``: ``local`` (in-process
``LocalMaster``) or an ``http://host:port`` / ``zk://`` v1 master, with the reference's credential
rules.
"""
from __future__ import annotations

import gc
import logging
import os
import sys
from typing import Callable, Optional, Set

from dcos_commons_amd.dcos import capabilities as caps
from dcos_commons_amd.http import endpoint_utils
from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.scheduler.plan.elements import DefaultPlan
from dcos_commons_amd.scheduler.plan.managers import DefaultPlanCoordinator, DefaultPlanManager
from dcos_commons_amd.scheduler.plan.strategy import SerialStrategy
from dcos_commons_amd.state.framework_store import FrameworkStore
from dcos_commons_amd.storage.persister_utils import clear_all_data

from .framework_scheduler import FrameworkScheduler
from .process_exit import ProcessExit

LOGGER = logging.getLogger(__name__)
TWO_WEEK_SEC = 2 * 7 * 24 * 60 * 60
API_SERVER_WAIT_S = 5.0   # SDK_EARLY_SUBSCRIBE: how long early offers wait for the API server
Cap = P.FrameworkInfo.Capability


class FrameworkRunner:
    def __init__(self, scheduler_config, framework_config, using_gpus: bool, using_regions: bool,
                 driver_factory: Optional[Callable] = None):
        self.scheduler_config = scheduler_config
        self.framework_config = framework_config
        self.using_gpus = using_gpus
        self.using_regions = using_regions
        self.driver_factory = driver_factory
        self.api_server = None
        self.framework_scheduler: Optional[FrameworkScheduler] = None
        self.driver = None

    def resource_roles(self) -> Set[str]:
        roles = {self.framework_config.role}
        roles.update(self.framework_config.pre_reserved_roles)
        if self.scheduler_config.enable_role_migration():  # both the legacy and the group (quota) role
            roles.add(self.framework_config.non_namespaced_role())
            ns = self.framework_config.namespaced_role()
            if ns is not None:
                roles.add(ns)
        return roles

    def get_framework_info(self, framework_id: Optional[P.FrameworkID]) -> P.FrameworkInfo:
        fc = self.framework_config
        info = P.FrameworkInfo(name=fc.framework_name, principal=fc.principal, user=fc.user,
                               failover_timeout=TWO_WEEK_SEC, checkpoint=True)
        if framework_id is not None:
            info.id.CopyFrom(framework_id)
        roles = self.resource_roles()
        if len(roles) > 1:
            info.capabilities.add(type=Cap.MULTI_ROLE)
            info.roles.extend(sorted(roles))
        else:
            info.role = fc.role
        if fc.web_url:
            info.webui_url = fc.web_url
        c = caps.get_instance()
        if c.supports_partition_awareness:
            info.capabilities.add(type=Cap.PARTITION_AWARE)
        if self.using_gpus and c.supports_gpu_resource:
            info.capabilities.add(type=Cap.GPU_RESOURCES)
        if c.supports_pre_reserved_resources:
            info.capabilities.add(type=Cap.RESERVATION_REFINEMENT)
        if self.using_regions and c.supports_domains:
            info.capabilities.add(type=Cap.REGION_AWARE)
        return info

    def _default_driver_factory(self):
        from .scheduler_driver_factory import default_driver_factory

        return default_driver_factory(self.scheduler_config)

    def start(self, persister, client, block: bool = True):
        """Registers and (if ``block``) runs until the driver stops. Returns the driver otherwise."""
        if self.scheduler_config.is_uninstall_enabled() and FrameworkStore(persister).fetch_framework_id() is None:
            clear_all_data(persister)
            self._run_skeleton_scheduler(block)
            ProcessExit.exit(ProcessExit.DRIVER_EXITED)
            return None
        switch_s = self.scheduler_config.gil_switch_interval_s()
        if switch_s > 0:
            sys.setswitchinterval(switch_s)
        gen0 = self.scheduler_config.gc_gen0_threshold()
        if gen0 > 0:
            _, g1, g2 = gc.get_threshold()
            gc.set_threshold(gen0, g1, g2)
        cpus = self.scheduler_config.cpu_set()
        if cpus:
            try:
                os.sched_setaffinity(0, cpus)   # threads started from here on inherit it
            except (AttributeError, OSError) as e:
                LOGGER.warning("Unable to pin the scheduler to CPUs %s: %s", cpus, e)
        framework_store = FrameworkStore(persister)
        self.framework_scheduler = FrameworkScheduler(self.resource_roles(), self.scheduler_config, persister,
                                                      framework_store, client)
        hostname = endpoint_utils.to_scheduler_auto_ip_hostname(self.framework_config.framework_name,
                                                                self.scheduler_config)
        from dcos_commons_amd.http.server import ApiServer

        def start_api_server():
            self.api_server = ApiServer.start(self.scheduler_config, client.get_http_endpoints(),
                                              self.framework_scheduler.set_api_server_started,
                                              scheduler_hostname=hostname)

        early = self.scheduler_config.is_early_subscribe()
        if not early:
            start_api_server()
        info = self.get_framework_info(framework_store.fetch_framework_id())
        factory = self.driver_factory or self._default_driver_factory()
        self.driver = factory(self.framework_scheduler, info)
        prestart = self.scheduler_config.thread_prestart()
        if prestart == "before" or (prestart == "after" and block):
            self.framework_scheduler.prestart()
        if early:
            # SUBSCRIBE goes out first and the API server starts during the registration round
            # trip; offers that arrive before it is up wait for it instead of being declined
            self.framework_scheduler.api_server_wait_s = API_SERVER_WAIT_S
            self.driver.start()
            start_api_server()
        if not block:
            if not early:
                self.driver.start()
            if prestart == "after":
                self.framework_scheduler.prestart()
            return self.driver
        if early:
            self.driver.join()
        else:
            self.driver.run()
        self.api_server.join()
        ProcessExit.exit(ProcessExit.DRIVER_EXITED)
        return None

    register_and_run_framework = start

    def _run_skeleton_scheduler(self, block: bool) -> None:
        from dcos_commons_amd.http.resources import HealthResource, PlansResource
        from dcos_commons_amd.http.server import ApiServer

        pm = DefaultPlanManager.create_proceeding(DefaultPlan("deploy", [], SerialStrategy(), []))
        coordinator = DefaultPlanCoordinator([pm])
        self.api_server = ApiServer.start(self.scheduler_config, [PlansResource([pm]), HealthResource(coordinator)],
                                          lambda: LOGGER.info("Started trivially healthy API server."))
        if block:
            self.api_server.join()

    def stop(self) -> None:
        if self.framework_scheduler is not None:
            self.framework_scheduler.stop()
        if self.driver is not None:
            self.driver.stop(True)
        if self.api_server is not None:
            self.api_server.stop()
