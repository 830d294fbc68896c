"""Entry point that turns a ServiceSpec (or YAML) into a running scheduler.

Reference: sdk/.../scheduler/SchedulerRunner.java:30-140: check the schema version, configure
StatsD, build the FrameworkRunner (GPU capability if any pod asks for GPUs, region awareness),
build the scheduler and register/run it.
"""
from __future__ import annotations

from typing import Callable, Optional

from dcos_commons_amd import metrics
from dcos_commons_amd.config.validate import service_requests_gpu_resources
from dcos_commons_amd.framework.framework_config import FrameworkConfig
from dcos_commons_amd.framework.framework_runner import FrameworkRunner
from dcos_commons_amd.scheduler.scheduler_builder import SchedulerBuilder
from dcos_commons_amd.state.schema_version_store import SchemaVersion, SchemaVersionStore


class SchedulerRunner:
    def __init__(self, builder: SchedulerBuilder, driver_factory: Optional[Callable] = None):
        self.builder = builder
        self.driver_factory = driver_factory
        self.framework_runner: Optional[FrameworkRunner] = None
        self.scheduler = None

    @staticmethod
    def from_raw_service_spec(raw, scheduler_config, config_template_dir=None, **kw) -> "SchedulerRunner":
        from dcos_commons_amd.specification.yaml.mappers import ServiceSpecGenerator

        spec = ServiceSpecGenerator(raw, scheduler_config, config_template_dir).build()
        return SchedulerRunner(SchedulerBuilder(spec, scheduler_config).set_plans_from(raw), **kw)

    @staticmethod
    def from_service_spec(spec, scheduler_config, **kw) -> "SchedulerRunner":
        return SchedulerRunner(SchedulerBuilder(spec, scheduler_config), **kw)

    @staticmethod
    def from_scheduler_builder(builder: SchedulerBuilder, **kw) -> "SchedulerRunner":
        return SchedulerRunner(builder, **kw)

    def run(self, block: bool = True):
        cfg = self.builder.scheduler_config
        spec = self.builder.original_service_spec
        persister = self.builder.persister
        SchemaVersionStore(persister).check(SchemaVersion.SINGLE_SERVICE)
        metrics.configure_statsd(cfg)
        self.framework_runner = FrameworkRunner(
            cfg, FrameworkConfig.from_service_spec(spec, cfg.service_namespace()),
            service_requests_gpu_resources(spec), self.builder.is_region_awareness_enabled(),
            driver_factory=self.driver_factory)
        self.scheduler = self.builder.build()
        if block:
            from dcos_commons_amd.framework.process_exit import install_signal_handlers

            install_signal_handlers()
        return self.framework_runner.start(persister, self.scheduler, block=block)

    def stop(self) -> None:
        if self.framework_runner is not None:
            self.framework_runner.stop()
