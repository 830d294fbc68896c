"""Scheduler flag system: ~45 environment variables with defaults.

Reference: sdk/.../scheduler/SchedulerConfig.java:56-666. The defaults here are identical to the
reference; MI355X-specific additions are prefixed ``SDK_`` and documented inline.
"""
from __future__ import annotations

from typing import Dict, Optional

from dcos_commons_amd.framework.env_store import EnvStore
from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.state.goal_state_override import PAUSE_COMMAND

DEFAULT_SCHEDULER_ROLE = "slave_public"
MESOS_API_VERSION_V1 = "V1"


def _scalar(v: float) -> P.Value:
    val = P.Value(type=P.Value.SCALAR)
    val.scalar.value = v
    return val


def parse_cpu_list(text: str) -> list:
    """``"0-3,8,10-11"`` -> ``[0, 1, 2, 3, 8, 10, 11]`` (Linux cpu-list syntax)."""
    cpus = set()
    for part in text.split(","):
        part = part.strip()
        if not part:
            continue
        lo, sep, hi = part.partition("-")
        a, b = int(lo), int(hi) if sep else int(lo)
        if a < 0 or b < a:
            raise ValueError(f"Invalid cpu range '{part}' in '{text}'")
        cpus.update(range(a, b + 1))
    if not cpus:
        raise ValueError(f"Empty cpu list '{text}'")
    return sorted(cpus)


class SchedulerConfig:
    _printed_build_info = False

    def __init__(self, env_store: Optional[EnvStore] = None):
        self.env = env_store or EnvStore.from_env()
        if not SchedulerConfig._printed_build_info:  # once per process (SchedulerConfig.java:322-324)
            SchedulerConfig._printed_build_info = True
            import json
            import logging

            logging.getLogger(__name__).info("Build information:\n%s", json.dumps(self.build_info(), indent=2))

    @staticmethod
    def from_env() -> "SchedulerConfig":
        return SchedulerConfig(EnvStore.from_env())

    @staticmethod
    def from_map(m: Dict[str, str]) -> "SchedulerConfig":
        return SchedulerConfig(EnvStore.from_map(m))

    @staticmethod
    def for_testing(**overrides) -> "SchedulerConfig":
        """Equivalent of the reference's SchedulerConfigTestUtils.getTestSchedulerConfig()."""
        env = {
            "PORT_API": "8080",
            "BOOTSTRAP_URI": "bootstrap-uri",
            "LIBMESOS_URI": "libmesos-uri",
            "JAVA_URI": "java-uri",
            "JAVA_HOME": "java-home",
            "PACKAGE_NAME": "test-package",
            "PACKAGE_VERSION": "1.0",
            "PACKAGE_BUILD_TIME_EPOCH_MS": "0",
            "LIBPROCESS_IP": "127.0.0.1",
            "DISABLE_DEADLOCK_EXIT": "true",
            # tests never share an on-disk state tree (or its lock) through the working directory
            "SDK_PERSISTER": "mem",
        }
        env.update({k: str(v) for k, v in overrides.items()})
        return SchedulerConfig(EnvStore.from_map(env))

    # timeouts
    def api_server_init_timeout_s(self) -> int:
        return self.env.get_optional_int("API_SERVER_TIMEOUT_S", 600)

    def multi_service_removal_timeout_s(self) -> int:
        return self.env.get_optional_int("SERVICE_REMOVAL_TIMEOUT_S", 600)

    def multi_service_reserve_discipline(self) -> int:
        return self.env.get_optional_int("RESERVE_DISCIPLINE", 0)

    def auth_token_refresh_threshold_s(self) -> int:
        return self.env.get_optional_int("AUTH_TOKEN_REFRESH_THRESHOLD_S", 30)

    # executor
    def executor_resources(self) -> Dict[str, P.Value]:
        return {
            "cpus": _scalar(self.env.get_optional_double("EXECUTOR_CPUS", 0.1)),
            "disk": _scalar(self.env.get_optional_double("EXECUTOR_DISK_MB", 256)),
            "mem": _scalar(self.env.get_optional_double("EXECUTOR_MEM_MB", 32)),
        }

    # identity / uris
    def api_server_port(self) -> int:
        return self.env.get_required_int("PORT_API")

    def bootstrap_uri(self) -> str:
        return self.env.get_optional("BOOTSTRAP_URI", "")

    def libmesos_uri(self) -> str:
        return self.env.get_optional("LIBMESOS_URI", "")

    def java_uri(self) -> str:
        return self.env.get_optional("JAVA_URI", "")

    def java_home(self) -> str:
        return self.env.get_optional("JAVA_HOME", "")

    def dcos_space(self) -> str:
        v = self.env.get_optional("DCOS_SPACE", None)
        if v is not None:
            return v
        return self.env.get_optional("MARATHON_APP_ID", "/")

    def scheduler_region(self) -> Optional[str]:
        return self.env.get_optional("SERVICE_REGION", None)

    def service_namespace(self) -> Optional[str]:
        if self.env.get_optional_boolean("MARATHON_APP_ENFORCE_GROUP_ROLE", False):
            return self.env.get_required("MESOS_ALLOCATION_ROLE")
        preferred = self.env.get_optional("MESOS_ALLOCATION_ROLE", None)
        if preferred is not None and preferred != DEFAULT_SCHEDULER_ROLE:
            return preferred
        return None

    def enable_role_migration(self) -> bool:
        return self.env.get_optional_boolean("ENABLE_ROLE_MIGRATION", False)

    def secrets_namespace(self, service_name: str) -> str:
        ns = self.dcos_space().lstrip("/")
        return ns if ns else service_name

    # switches
    def is_state_cache_enabled(self) -> bool:
        return not self.env.is_present("DISABLE_STATE_CACHE")

    def is_deadlock_exit_enabled(self) -> bool:
        return not self.env.is_present("DISABLE_DEADLOCK_EXIT")

    def is_suppress_enabled(self) -> bool:
        return not self.env.is_present("DISABLE_SUPPRESS")

    def is_uninstall_enabled(self) -> bool:
        return self.env.is_present("SDK_UNINSTALL")

    def use_legacy_unneeded_task_kills(self) -> bool:
        return self.env.is_present("USE_LEGACY_KILL_UNNEEDED_TASKS")

    def is_side_channel_active(self) -> bool:
        return self.env.is_present("DCOS_SERVICE_ACCOUNT_CREDENTIAL")

    def side_channel_credential(self) -> Optional[str]:
        return self.env.get_optional("DCOS_SERVICE_ACCOUNT_CREDENTIAL", None)

    def dcos_auth_token_provider(self):
        """Cached IAM token provider for the service account (SchedulerConfig.java:484-523)."""
        from dcos_commons_amd.dcos.clients import ConstantTokenProvider, token_provider_from_service_account

        static = self.env.get_optional("SDK_DCOS_AUTH_TOKEN", None)
        if static:
            return ConstantTokenProvider(static)
        return token_provider_from_service_account(self.env.get_required("DCOS_SERVICE_ACCOUNT_CREDENTIAL"),
                                                   self.auth_token_refresh_threshold_s())

    # statsd
    def statsd_poll_interval_s(self) -> int:
        return self.env.get_optional_long("STATSD_POLL_INTERVAL_S", 10)

    def statsd_host(self) -> Optional[str]:
        return self.env.get_optional("STATSD_UDP_HOST", None)

    def statsd_port(self) -> Optional[int]:
        v = self.env.get_optional("STATSD_UDP_PORT", None)
        return int(v) if v else None

    # mesos
    def mesos_api_version(self) -> str:
        return self.env.get_optional("MESOS_API_VERSION", MESOS_API_VERSION_V1)

    def mesos_master_url(self) -> str:
        """MI355X build: the v1 HTTP endpoint of the master (``SDK_MESOS_MASTER``)."""
        return self.env.get_optional("SDK_MESOS_MASTER", "http://leader.mesos:5050")

    def mesos_content_type(self) -> str:
        """``protobuf`` (default) or ``json`` body encoding on the v1 scheduler API."""
        v = self.env.get_optional("SDK_MESOS_CONTENT_TYPE", "protobuf").lower()
        return "application/json" if v == "json" else "application/x-protobuf"

    def is_driver_reconnect(self) -> bool:
        """MI355X build: resubscribe after a lost event stream instead of exiting (reference exits)."""
        return self.env.get_optional_boolean("SDK_DRIVER_RECONNECT", False)

    def is_async_mesos_calls(self) -> bool:
        """Mesos v1 calls (ACCEPT, ACKNOWLEDGE, KILL, REVIVE, ...) are POSTed in order by one sender
        thread and the caller does not wait for the HTTP answer (``SDK_ASYNC_MESOS_CALLS``, default
        on), as the reference's libprocess-backed driver does; off: each call is a synchronous
        request whose failure raises in the caller."""
        return self.env.get_optional_boolean("SDK_ASYNC_MESOS_CALLS", True)

    def mesos_credential(self):
        """Principal + secret from ``SDK_MESOS_PRINCIPAL``/``SDK_MESOS_SECRET`` (tools and tests that
        build a driver by hand; the scheduler itself uses SchedulerDriverFactory's rules)."""
        principal = self.env.get_optional("SDK_MESOS_PRINCIPAL", "")
        if not principal:
            return None
        from dcos_commons_amd.mesos import protos as P

        return P.Credential(principal=principal, secret=self.env.get_optional("SDK_MESOS_SECRET", ""))

    def pause_override_cmd(self) -> str:
        return self.env.get_optional("PAUSE_OVERRIDE_CMD", PAUSE_COMMAND)

    def autoip_tld(self) -> str:
        return self.env.get_optional("SERVICE_TLD", "autoip.dcos.thisdcos.directory")

    def vip_tld(self) -> str:
        return self.env.get_optional("VIP_TLD", "l4lb.thisdcos.directory")

    def marathon_name(self) -> str:
        return self.env.get_optional("MARATHON_NAME", "marathon")

    def implicit_reconcile_delay_ms(self) -> int:
        return self.env.get_optional_long("IMPLICIT_RECONCILIATION_DELAY_MS", 0)

    def implicit_reconcile_period_ms(self) -> int:
        return self.env.get_optional_long("IMPLICIT_RECONCILIATION_PERIOD_MS", 60 * 60 * 1000)

    def is_region_awareness_enabled(self) -> bool:
        return self.env.get_optional_boolean("ALLOW_REGION_AWARENESS", True)

    def scheduler_ip(self) -> str:
        return self.env.get_optional("LIBPROCESS_IP", "127.0.0.1")

    # backoff (reference plan/backoff/Backoff.java:17-50)
    def is_backoff_enabled(self) -> bool:
        return self.env.get_optional_boolean("ENABLE_BACKOFF", False)

    def backoff_factor(self) -> float:
        return self.env.get_optional_double("FRAMEWORK_BACKOFF_FACTOR", 1.15)

    def initial_backoff_s(self) -> int:
        return self.env.get_optional_int("FRAMEWORK_INITIAL_BACKOFF", 60)

    def max_launch_delay_s(self) -> int:
        return self.env.get_optional_int("FRAMEWORK_MAX_LAUNCH_DELAY", 300)

    # offer processing cadence (reference OfferProcessor.java:46 hard-codes 5 s; the
    # event-driven MI355X build wakes immediately on offers/status updates and uses this only
    # as the idle poll interval).
    def offer_wait_s(self) -> float:
        return self.env.get_optional_double("SDK_OFFER_WAIT_S", 5.0)

    def gil_switch_interval_s(self) -> float:
        """Interpreter thread switch interval for the scheduler process (``SDK_GIL_SWITCH_INTERVAL_MS``;
        default 0 = keep the interpreter's 5 ms). The offer loop, the status path and the API threads
        share one interpreter lock. A longer interval lets an offer cycle finish before a status is
        handled; unpinned, that took an 8-agent deploy from 58 to 41 ms on a slow CPU, but with the
        process pinned to a few cores (bench.py) it only added tail latency (8-pod deploys with
        22-37 ms outliers against <= 16 ms at 5 ms, profiles/ab_gil_interval_pinned_r03.txt)."""
        return float(self.env.get_optional("SDK_GIL_SWITCH_INTERVAL_MS", "0") or 0) / 1000.0

    def gc_gen0_threshold(self) -> int:
        """Allocations between young-generation collections of the cyclic garbage collector
        (``SDK_GC_GEN0_THRESHOLD``; 0 = keep the interpreter's 700). Protobuf-heavy offer cycles
        allocate tens of thousands of objects; each collection pauses whichever thread is
        allocating, which is often the offer loop. 20000 on the box (interleaved, 20 reps): 8-pod
        deploy 10.1 -> 9.5 ms, 1-pod deploy 4.6 -> 4.4 ms (profiles/ab_gc_gen0_threshold_box.txt)."""
        return self.env.get_optional_int("SDK_GC_GEN0_THRESHOLD", 20000)

    def cpu_set(self) -> Optional[list]:
        """CPUs the scheduler process runs on (``SDK_CPU_SET``, a Linux cpu list such as ``4-7`` or
        ``2,3,8-9``; unset = wherever the OS puts it). Applied when the framework starts, so every
        scheduler thread inherits it: the offer loop, status path and API threads hand work to each
        other, and on a few warm cores those hand-offs do not wait for an idle core to wake
        (bench.py pins its ranks the same way: deploy 4.2-5.1 -> 2.8 ms on the box)."""
        v = self.env.get_optional("SDK_CPU_SET", "").strip()
        return parse_cpu_list(v) if v else None

    def is_revive_only_unmatched(self) -> bool:
        """Skip the REVIVE that new work asked for when the same offer cycle matched all of it
        (``SDK_REVIVE_ONLY_UNMATCHED``; reference: revive on every work-set change). The revive
        would only bring this cycle's leftovers back for another evaluation pass. Applies only with
        ``SDK_OFFER_HOLD_S`` > 0: without held offers the leftovers are declined for an hour, and
        the revive is what clears those decline filters for a later relaunch of the same step."""
        return self.env.get_optional_boolean("SDK_REVIVE_ONLY_UNMATCHED", True)

    def is_event_driven(self) -> bool:
        """Wake the offer loop on every status update (reference: poll only)."""
        return self.env.get_optional_boolean("SDK_EVENT_DRIVEN", True)

    def status_cycle_wait_s(self) -> float:
        """How long a status update read from a network driver waits for a running offer cycle
        to finish before it is handled (``SDK_STATUS_CYCLE_WAIT_MS``; 0 = handle it at once, as the
        reference's driver callbacks do). See ``OfferProcessor.wait_cycle_idle``."""
        return self.env.get_optional_double("SDK_STATUS_CYCLE_WAIT_MS", 100.0) / 1000.0

    def is_offer_prewarm(self) -> bool:
        """Build the first evaluation's templates between registration and the first offers
        (``SDK_OFFER_PREWARM``; ``DefaultScheduler.prewarm``). Off by default: on the box it took
        the first evaluation 0.55 -> 0.37 ms but delayed handling the first offers by more, 1 pod
        2.02 -> 2.27 ms (profiles/prewarm_window_ab_r06_box.txt)."""
        return self.env.get_optional_boolean("SDK_OFFER_PREWARM", False)

    def thread_prestart(self) -> str:
        """When the offer-loop and implicit-reconciler threads are created (``SDK_THREAD_PRESTART``;
        ``FrameworkScheduler.prestart``): ``before`` SUBSCRIBE goes out, ``after`` it (a
        non-blocking driver: thread start-up overlaps the registration round trip), or ``false``
        (default): in the ``registered`` callback, as the reference starts its offer loop. Not
        adopted: on the box all three were within the spread, 1 pod 1.94-1.97 ms and 8 pods
        5.26-5.29 ms best of three (profiles/prestart_ab_r06_box.txt)."""
        v = self.env.get_optional("SDK_THREAD_PRESTART", "false").strip().lower()
        return {"true": "before", "1": "before", "0": "false", "no": "false"}.get(v, v)

    def is_early_subscribe(self) -> bool:
        """Send SUBSCRIBE before starting the API server, which then starts during the registration
        round trip (``SDK_EARLY_SUBSCRIBE``; ``FrameworkRunner.start``). The reference starts the
        server first and declines offers that arrive before it is up. Not adopted: no difference on
        the box (1 pod 2.01 vs 2.02 ms; profiles/early_subscribe_ab_r06_box.txt)."""
        return self.env.get_optional_boolean("SDK_EARLY_SUBSCRIBE", False)

    def offer_hold_s(self) -> float:
        """Hold unused offers this long while WORKING instead of declining them for 1 h
        (0 = reference behaviour: long decline + rate-limited revive)."""
        return self.env.get_optional_double("SDK_OFFER_HOLD_S", 10.0)

    def revive_interval_s(self) -> float:
        """Minimum spacing of REVIVE calls. The reference hard-codes 5 s (TokenBucket.java:18-24);
        the 256-token budget (+1 per 256 s) still bounds the sustained rate, so a 1 s burst spacing
        costs the master little and takes up to 4 s off every recovery that needs a revive."""
        return self.env.get_optional_double("SDK_REVIVE_INTERVAL_S", 1.0)

    def revive_burst_interval_s(self) -> float:
        """REVIVE spacing while the revive token bucket is more than half full (a burst of new
        candidate steps, e.g. a pod relaunching in place after its ONCE task finished, gets its
        offers within one allocation instead of waiting out ``SDK_REVIVE_INTERVAL_S``). Clamped
        to the revive interval; the reference has no burst regime."""
        return min(self.env.get_optional_double("SDK_REVIVE_BURST_INTERVAL_S", 0.05), self.revive_interval_s())

    def is_reservation_gc_on_all_offers(self) -> bool:
        """Release stale reservations from every offer, idle or not (reference: unused offers
        while WORKING only)."""
        return self.env.get_optional_boolean("SDK_RESERVATION_GC_ALL_OFFERS", True)

    def is_merge_agent_offers(self) -> bool:
        """Evaluate all outstanding offers of one agent as a single offer and ACCEPT them together
        (reference: every offer on its own)."""
        return self.env.get_optional_boolean("SDK_MERGE_AGENT_OFFERS", True)

    def is_fast_unsuppress(self) -> bool:
        """First REVIVE after a SUPPRESS skips the burst spacing (reference: never)."""
        return self.env.get_optional_boolean("SDK_FAST_UNSUPPRESS", True)

    def is_stream_launches(self) -> bool:
        """ACCEPT each matched step's launch immediately instead of after the whole offer cycle
        (reference: one batch of ACCEPTs at the end of the cycle)."""
        return self.env.get_optional_boolean("SDK_STREAM_LAUNCHES", True)

    def pipeline_launch_writes(self) -> Optional[bool]:
        """Overlap each streamed step's write-ahead record (its TaskInfos, in ZooKeeper) with the
        evaluation of the next steps, writing what has queued up in one transaction and sending
        the ACCEPTs in step order once it is durable (``SDK_PIPELINE_LAUNCH_WRITES``; unset: on
        when the persister is remote). No reference counterpart: the reference records a cycle's
        launches in one write after evaluating all of it, and its launches wait for that."""
        v = self.env.get_optional("SDK_PIPELINE_LAUNCH_WRITES", "")
        return None if v in ("", "auto") else v.lower() in ("1", "true", "yes")

    def launch_reconcile_s(self) -> float:
        """Explicitly reconcile a launch that still has no status after this many seconds, e.g.
        because its ACCEPT was lost (0 = reference behaviour: wait for the next scheduler
        restart)."""
        return self.env.get_optional_double("SDK_LAUNCH_RECONCILE_S", 30.0)

    def is_unknown_as_lost(self) -> bool:
        """Trust the master's "never heard of this task": a reconciliation TASK_UNKNOWN is handled as
        TASK_LOST so the task is recovered (in place: a TRANSIENT recovery on the task's existing
        reservations), and a *first-footprint* launch (stored TaskInfo labelled
        ``launch_new_footprint``, i.e. every reservation it references was created by that launch)
        that the master reports LOST/DROPPED while our only record is the write-ahead STAGING
        status is relaunched with fresh reservations. An in-place relaunch never is: its
        reservations and volumes exist regardless of the lost ACCEPT (reference: the UNKNOWN status
        is stored and never recovered, and a lost first launch waits forever for reservations that
        were never made)."""
        return self.env.get_optional_boolean("SDK_UNKNOWN_AS_LOST", True)

    def implicit_reconcile_delay_s(self) -> float:
        return self.implicit_reconcile_delay_ms() / 1000.0

    def implicit_reconcile_period_s(self) -> float:
        return self.implicit_reconcile_period_ms() / 1000.0

    def package_build_time_ms(self) -> int:
        return self.env.get_optional_int("PACKAGE_BUILD_TIME_EPOCH_MS", 0)

    def build_info(self) -> Dict[str, str]:
        """Reference SchedulerConfig.getBuildInfo (SchedulerConfig.java:655-665): package identity
        plus the SDK's own build stamp (``sdk_build_info``), served by the multi-service
        ``/v1/health`` and logged once per process."""
        from dcos_commons_amd.utils import sdk_build_info as B

        return {
            "PACKAGE_NAME": self.env.get_optional("PACKAGE_NAME", ""),
            "PACKAGE_VERSION": self.env.get_optional("PACKAGE_VERSION", ""),
            "PACKAGE_BUILT_AT": B.iso_instant(self.package_build_time_ms()),
            "SDK_NAME": B.NAME,
            "SDK_VERSION": B.VERSION,
            "SDK_GIT_SHA": B.git_sha(),
            "SDK_BUILT_AT": B.iso_instant(B.build_time_ms()),
        }
