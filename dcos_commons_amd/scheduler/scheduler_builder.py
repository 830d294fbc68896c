"""Builds a service scheduler from a ServiceSpec.

Reference: sdk/.../scheduler/SchedulerBuilder.java:77-744. Injects the region placement rule,
picks the Uninstall or Default scheduler, runs the config update + validators, generates plans
(YAML or the default deploy plan), replaces ``deploy`` with the YAML ``update`` plan once deploy
has completed (:644), surfaces validation errors on the deploy plan, and builds the recovery
manager (Timed vs Never failure monitor), optional decommission manager and the coordinator.
"""
from __future__ import annotations

import logging
from dataclasses import replace
from typing import Dict, List, Optional

from dcos_commons_amd.config import validate as V
from dcos_commons_amd.config.configuration_updater import DefaultConfigurationUpdater
from dcos_commons_amd.dcos import capabilities
from dcos_commons_amd.framework.process_exit import ProcessExit
from dcos_commons_amd.http import endpoint_utils
from dcos_commons_amd.offer import constants
from dcos_commons_amd.offer.evaluate import placement as pl
from dcos_commons_amd.scheduler.decommission import DecommissionPlanFactory
from dcos_commons_amd.scheduler.default_scheduler import DefaultScheduler
from dcos_commons_amd.scheduler.plan.elements import DefaultPlan, get_launchable_tasks
from dcos_commons_amd.scheduler.plan.factories import (
    DefaultPhaseFactory,
    DefaultStepFactory,
    DeployPlanFactory,
    PlanGenerator,
)
from dcos_commons_amd.scheduler.plan.managers import (
    DecommissionPlanManager,
    DefaultPlanCoordinator,
    DefaultPlanManager,
)
from dcos_commons_amd.scheduler.recovery import (
    DefaultRecoveryPlanManager,
    NeverFailureMonitor,
    TimedFailureMonitor,
)
from dcos_commons_amd.offer.task_utils import has_tasks_with_tls
from dcos_commons_amd.scheduler.uninstall import UninstallScheduler
from dcos_commons_amd.specification.specs import ServiceSpec, loopback_check
from dcos_commons_amd.state import state_store_utils
from dcos_commons_amd.state.config_store import ConfigStore, ConfigStoreException
from dcos_commons_amd.state.framework_store import FrameworkStore
from dcos_commons_amd.state.state_store import StateStore
from dcos_commons_amd.storage.persister import Persister


class SchedulerBuilder:
    def __init__(self, service_spec: ServiceSpec, scheduler_config, persister: Optional[Persister] = None):
        self.original_service_spec = service_spec
        self.scheduler_config = scheduler_config
        if persister is None:
            from dcos_commons_amd.storage.factory import persister_for_service

            persister = persister_for_service(service_spec, scheduler_config)
        self.persister = persister
        self.yaml_plans: Dict[str, dict] = {}
        self.endpoint_producers: Dict[str, object] = {}
        self.custom_config_validators: List = []
        self.custom_resources: List = []
        self.recovery_plan_overrider_factory = None
        self.plan_customizer = None
        self.multi_service_framework_name: Optional[str] = None
        self.region_awareness_enabled = False
        self.tls_stage_factory = None
        self.logger = logging.getLogger(__name__)

    # -- fluent setters ----------------------------------------------------------------
    def set_custom_resources(self, resources) -> "SchedulerBuilder":
        self.custom_resources = list(resources)
        return self

    def set_custom_config_validators(self, validators) -> "SchedulerBuilder":
        self.custom_config_validators = list(validators)
        return self

    def set_endpoint_producer(self, name: str, producer) -> "SchedulerBuilder":
        self.endpoint_producers[name] = producer
        return self

    def set_plans_from(self, raw_service_spec) -> "SchedulerBuilder":
        if raw_service_spec.plans:
            self.yaml_plans = dict(raw_service_spec.plans)
        return self

    def set_recovery_manager_factory(self, factory) -> "SchedulerBuilder":
        self.recovery_plan_overrider_factory = factory
        return self

    def set_plan_customizer(self, customizer) -> "SchedulerBuilder":
        self.plan_customizer = customizer
        return self

    def with_single_region_constraint(self) -> "SchedulerBuilder":
        self.region_awareness_enabled = True
        return self

    def enable_multi_service(self, framework_name: str) -> "SchedulerBuilder":
        self.multi_service_framework_name = framework_name
        return self

    def set_tls_stage_factory(self, factory) -> "SchedulerBuilder":
        self.tls_stage_factory = factory
        return self

    def is_region_awareness_enabled(self) -> bool:
        return self.region_awareness_enabled or self.scheduler_config.is_region_awareness_enabled()

    # -- build ---------------------------------------------------------------------------
    def _with_region_rules(self, spec: ServiceSpec) -> ServiceSpec:
        if not capabilities.get_instance().supports_domains:
            return spec
        region = self.scheduler_config.scheduler_region()
        if self.is_region_awareness_enabled() and region:
            rule = pl.RegionRuleFactory.require(pl.ExactMatcher.create(region))
        else:
            rule = pl.IsLocalRegionRule()
        pods = []
        for p in spec.pods:
            if pl.references_region(p):
                pods.append(p)
            else:
                merged = pl.AndRule([rule, p.placement_rule]) if p.placement_rule is not None else rule
                pods.append(replace(p, placement_rule=merged))
        return replace(spec, pods=tuple(pods), region=region if region else spec.region)

    def build(self):
        namespace = self.original_service_spec.name if self.multi_service_framework_name else None
        spec = self._with_region_rules(self.original_service_spec)
        state_store = StateStore(self.persister, namespace)
        config_store = ConfigStore(loopback_check(spec), self.persister, namespace)
        framework_store = FrameworkStore(self.persister)
        if self.scheduler_config.is_uninstall_enabled():
            return UninstallScheduler(spec, state_store, config_store, self.scheduler_config, self.plan_customizer,
                                      namespace, framework_store)
        if state_store_utils.is_uninstalling(state_store):
            if self.multi_service_framework_name:
                return UninstallScheduler(spec, state_store, config_store, self.scheduler_config,
                                          self.plan_customizer, namespace, framework_store)
            self.logger.error("Service has been previously told to uninstall, this cannot be reversed. "
                              "Reenable the uninstall flag to complete the process.")
            ProcessExit.exit(ProcessExit.SCHEDULER_ALREADY_UNINSTALLING)
        try:
            return self._default_scheduler(spec, framework_store, state_store, config_store, namespace)
        except ConfigStoreException as e:
            self.logger.error("Failed to construct scheduler: %s", e)
            ProcessExit.exit(ProcessExit.INITIALIZATION_FAILURE, e)
            return None

    def _has_role_changed(self, config_store, spec) -> bool:
        try:
            tid = config_store.get_target_config()
        except ConfigStoreException:
            return False
        return config_store.fetch(tid).role != spec.role

    def _default_scheduler(self, spec, framework_store, state_store, config_store, namespace):
        completed = state_store_utils.get_deployment_was_completed(state_store)
        role_changed = self._has_role_changed(config_store, spec)
        validators = V.get_validators(self.scheduler_config) + V.get_role_validators(role_changed, completed) + \
            list(self.custom_config_validators)
        result = DefaultConfigurationUpdater(state_store, config_store, validators, namespace).update_configuration(spec)
        if result.errors:
            self.logger.warning("Failed to update configuration due to validation errors: %s", result.errors)
            spec = config_store.fetch(config_store.get_target_config())
        plans = self._plans(state_store, config_store, spec, namespace)
        plans = self.select_deploy_plan(plans, completed)
        deploy = self._deploy_plan(plans)
        if deploy is None:
            raise ValueError(f"No deploy plan provided: {plans}")
        errors = [str(e) for e in result.errors]
        if errors:
            new_deploy = DefaultPlan(deploy.get_name(), deploy.get_children(), deploy.get_strategy(), errors)
            plans = [new_deploy] + [p for p in plans if not p.is_deploy_plan()]
            deploy = new_deploy
        deploy_pm = DefaultPlanManager.create_proceeding(deploy)
        recovery_pm = self._recovery_plan_manager(spec, state_store, config_store, plans, namespace)
        decom = DecommissionPlanFactory(spec, state_store, namespace)
        managers = [deploy_pm, recovery_pm]
        if decom.get_plan() is not None:
            managers.append(DecommissionPlanManager(decom.get_plan(), decom.get_resource_steps(),
                                                    decom.get_tasks_to_decommission()))
        managers.extend(DefaultPlanManager.create_interrupted(p) for p in plans if not p.is_deploy_plan())
        coordinator = DefaultPlanCoordinator(managers, namespace)
        if self.multi_service_framework_name:
            url_factory = endpoint_utils.template_url_factory(self.multi_service_framework_name,
                                                              self.scheduler_config, prefix=spec.name)
        else:
            url_factory = endpoint_utils.template_url_factory(spec.name, self.scheduler_config)
        tls_factory = self.tls_stage_factory
        if tls_factory is None and has_tasks_with_tls(spec):
            # OfferEvaluator.java:287: the TLS stage builder exists only when some task wants TLS
            from dcos_commons_amd.offer.evaluate.stages import TLSEvaluationStage

            tls_factory = TLSEvaluationStage.Builder(spec.name, self.scheduler_config)
        return DefaultScheduler(spec, self.scheduler_config, namespace, self.custom_resources, coordinator,
                                self.plan_customizer, framework_store, state_store, config_store, url_factory,
                                self.endpoint_producers, tls_factory)

    def _recovery_plan_manager(self, spec, state_store, config_store, plans, namespace):
        overriders = []
        if self.recovery_plan_overrider_factory is not None:
            overriders.append(self.recovery_plan_overrider_factory.create(state_store, plans))
        if spec.replacement_failure_policy is not None:
            monitor = TimedFailureMonitor(spec.replacement_failure_policy.permanent_failure_timeout_mins * 60.0,
                                          state_store, config_store)
        else:
            monitor = NeverFailureMonitor()
        return DefaultRecoveryPlanManager(state_store, config_store, get_launchable_tasks(plans), monitor, namespace,
                                          overriders)

    def _plans(self, state_store, config_store, spec, namespace) -> List[DefaultPlan]:
        step_factory = DefaultStepFactory(config_store, state_store, namespace)
        if self.yaml_plans:
            gen = PlanGenerator(step_factory)
            return [gen.generate(raw, name, spec.pods) for name, raw in self.yaml_plans.items()]
        if config_store.list():
            factory = DeployPlanFactory(DefaultPhaseFactory(step_factory))
            return [factory.get_plan(config_store.fetch(config_store.get_target_config()))]
        return []

    @staticmethod
    def _deploy_plan(plans):
        deploys = [p for p in plans if p.is_deploy_plan()]
        if len(deploys) > 1:
            raise ValueError(f"Found multiple deploy plans: {deploys}")
        return deploys[0] if deploys else None

    @staticmethod
    def select_deploy_plan(plans, has_completed_deployment: bool):
        update = next((p for p in plans if p.get_name() == constants.UPDATE_PLAN_NAME), None)
        if update is None:
            return plans
        if not has_completed_deployment:
            return [p for p in plans if p.get_name() != constants.UPDATE_PLAN_NAME]
        out = [p for p in plans if not p.is_deploy_plan() and p.get_name() != constants.UPDATE_PLAN_NAME]
        out.append(DefaultPlan(constants.DEPLOY_PLAN_NAME, update.get_children(), update.get_strategy(), []))
        return out
