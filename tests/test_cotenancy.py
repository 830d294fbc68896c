"""Co-tenancy bound of offer holding (``SDK_OFFER_HOLD_S``).

The scheduler holds offers it cannot use yet (instead of declining them for an hour, as the
reference does) so that a plan that advances can use them at once. While it holds them, no other
framework is offered those resources. The bound: another framework obtains resources the SDK
scheduler holds within ``hold_s`` plus one allocation interval of the scheduler receiving them,
after which the SDK's decline filter keeps them away from it (README, "Co-tenancy")."""
import os
import threading
import time

from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.mesos.local_master import AgentSpec, LocalMaster, LocalSchedulerDriver
from dcos_commons_amd.scheduler.scheduler_builder import SchedulerBuilder
from dcos_commons_amd.scheduler.scheduler_config import SchedulerConfig
from dcos_commons_amd.scheduler.scheduler_runner import SchedulerRunner
from dcos_commons_amd.specification.yaml.mappers import ServiceSpecGenerator
from dcos_commons_amd.specification.yaml.raw import RawServiceSpec
from dcos_commons_amd.storage.mem_persister import MemPersister

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SPECS = os.path.join(ROOT, "frameworks", "helloworld", "specs")
HOLD_S = 1.0
ALLOCATION_S = 0.05


class _Tenant:
    """A second framework on the same master: records when it is first offered cpus."""

    def __init__(self):
        self.first_cpus = None
        self.got = threading.Event()

    def registered(self, driver, fid, info):
        pass

    def resource_offers(self, driver, offers):
        cpus = sum(r.scalar.value for o in offers for r in o.resources if r.name == "cpus")
        if cpus > 0 and self.first_cpus is None:
            self.first_cpus = (time.monotonic(), cpus)
            self.got.set()
        driver.decline_offers([o.id for o in offers], P.Filters(refuse_seconds=3600))

    def status_update(self, driver, status):
        pass


def test_a_second_framework_gets_held_resources_within_hold_plus_one_allocation():
    env = dict(FRAMEWORK_NAME="hello-world", FRAMEWORK_PRINCIPAL="hw-principal", FRAMEWORK_USER="nobody",
               HELLO_COUNT="1", HELLO_PLACEMENT="", HELLO_CPUS="4", HELLO_MEM="256", HELLO_DISK="25",
               SLEEP_DURATION="1000", WORLD_COUNT="0", WORLD_PLACEMENT="", WORLD_CPUS="0.1", WORLD_MEM="64",
               WORLD_DISK="25", WORLD_READINESS_CHECK_INTERVAL="5", WORLD_READINESS_CHECK_DELAY="0",
               WORLD_READINESS_CHECK_TIMEOUT="10")
    cfg = SchedulerConfig.for_testing(PORT_API="0", SDK_OFFER_HOLD_S=str(HOLD_S), SDK_OFFER_WAIT_S="0.2")
    raw = RawServiceSpec.new_builder(os.path.join(SPECS, "svc.yml")).set_env(env).build()
    spec = ServiceSpecGenerator(raw, cfg, SPECS, env).build()
    master = LocalMaster(allocation_interval_s=ALLOCATION_S)
    master.add_agent(AgentSpec(hostname="only-agent", cpus=2, mem=4096, disk=20000))   # too small for hello
    runner = SchedulerRunner(SchedulerBuilder(spec, cfg, MemPersister()).set_plans_from(raw),
                             driver_factory=lambda s, i: LocalSchedulerDriver(master, s, i))
    tenant_driver = None
    try:
        runner.run(block=False)
        op = runner.framework_runner.framework_scheduler.offer_processor
        deadline = time.monotonic() + 10
        while not op.held_offer_ids() and time.monotonic() < deadline:
            time.sleep(0.005)
        held_at = time.monotonic()
        assert op.held_offer_ids(), "the SDK scheduler never held the agent's offer"
        assert not runner.scheduler.get_plan("deploy").is_complete()     # working: hello cannot be placed

        tenant = _Tenant()
        tenant_driver = LocalSchedulerDriver(master, tenant, P.FrameworkInfo(name="tenant", user="nobody",
                                                                             roles=["*"]))
        tenant_driver.start()
        assert tenant.got.wait(HOLD_S + 5), "the second framework never got the held cpus"
        waited = tenant.first_cpus[0] - held_at
        # everything the agent has was in the held offer: the tenant waits for the hold to end...
        assert waited > 0.5 * HOLD_S, waited
        # ...and then gets it at the next allocation (plus scheduling slack on a loaded machine)
        assert waited <= HOLD_S + ALLOCATION_S + 0.5, waited
        assert tenant.first_cpus[1] == 2.0
    finally:
        if tenant_driver is not None:
            tenant_driver.stop(failover=False)
        runner.stop()
        master.shutdown()
