"""Creates the scheduler driver: which master transport, which credential.

Reference: sdk/.../framework/SchedulerDriverFactory.java:27-202. The credential follows the
reference's rule: an explicit secret gives ``principal + secret``; otherwise DC/OS side-channel
auth (``DCOS_SERVICE_ACCOUNT_CREDENTIAL`` present) gives a principal-only credential; otherwise
none. Either kind of authentication needs a non-empty ``FrameworkInfo.principal``.

The reference then picks a V1 (HTTP) or V0 (libmesos JNI) Mesos client from
``MESOS_API_VERSION`` and the cluster's capabilities. There is no libmesos here: every remote
master is spoken to over the v1 HTTP scheduler API (``V1HttpSchedulerDriver``), so a V0 request
is logged and served by the v1 client. Side-channel credentials authenticate each call with the
service account's IAM token (``Authorization: token=<jwt>``, what DC/OS adminrouter expects); a
secret authenticates with HTTP Basic ``principal:secret``. ``SDK_MESOS_MASTER=local`` runs against
the in-process ``LocalMaster`` instead.
"""
from __future__ import annotations

import logging
from typing import Callable, Optional

from dcos_commons_amd.dcos import capabilities as caps
from dcos_commons_amd.mesos import protos as P

LOGGER = logging.getLogger(__name__)
MESOS_API_VERSION_V1 = "V1"


def _principal(framework_info: P.FrameworkInfo, auth_type: str) -> str:
    if not framework_info.principal:
        raise ValueError(f"Unable to create MesosSchedulerDriver for {auth_type} auth, FrameworkInfo lacks required "
                         f"principal: {framework_info}")
    return framework_info.principal


def get_credential(framework_info: P.FrameworkInfo, scheduler_config,
                   credential_secret: Optional[bytes] = None) -> Optional[P.Credential]:
    if credential_secret:
        LOGGER.info("Creating secret authenticated scheduler driver for framework[%s], credentialSecret[%d bytes]",
                    framework_info.name, len(credential_secret))
        secret = credential_secret.decode("utf-8") if isinstance(credential_secret, bytes) else str(credential_secret)
        return P.Credential(principal=_principal(framework_info, "secret"), secret=secret)
    if scheduler_config.is_side_channel_active():
        LOGGER.info("Creating sidechannel authenticated scheduler driver for framework[%s]", framework_info.name)
        return P.Credential(principal=_principal(framework_info, "sidechannel"))
    LOGGER.info("Creating unauthenticated scheduler driver for framework[%s]", framework_info.name)
    return None


def select_api_version(requested: str, capabilities=None) -> str:
    """What the reference would run (SchedulerDriverFactory.startInternalCustom): V1 only when
    requested and supported by the cluster, else V0."""
    c = capabilities or caps.get_instance()
    if requested == MESOS_API_VERSION_V1 and c.supports_v1_api_by_default:
        return MESOS_API_VERSION_V1
    return "V0"


class SchedulerDriverFactory:
    def create(self, scheduler, framework_info: P.FrameworkInfo, master_url: str, scheduler_config,
               credential_secret: Optional[bytes] = None):
        credential = get_credential(framework_info, scheduler_config, credential_secret)
        return self.create_internal(scheduler, framework_info, master_url, credential, scheduler_config)

    def create_internal(self, scheduler, framework_info, master_url, credential, scheduler_config):
        """Broken out so tests can substitute the transport (reference createInternal)."""
        version = select_api_version(scheduler_config.mesos_api_version())
        if version != MESOS_API_VERSION_V1:
            LOGGER.warning("Mesos %s API requested (MESOS_API_VERSION=%s): no libmesos in this build, using the v1 "
                           "HTTP scheduler API", version, scheduler_config.mesos_api_version())
        if master_url.startswith(("http://", "https://", "zk://")):
            from dcos_commons_amd.mesos.http_driver import V1HttpSchedulerDriver, resolve_master_url

            token_provider = None
            if credential is not None and not credential.secret and scheduler_config.is_side_channel_active():
                provider = scheduler_config.dcos_auth_token_provider()
                token_provider = provider.get_token
            return V1HttpSchedulerDriver(resolve_master_url(master_url), scheduler, framework_info,
                                         credential=credential, content_type=scheduler_config.mesos_content_type(),
                                         reconnect=scheduler_config.is_driver_reconnect(),
                                         token_provider=token_provider,
                                         async_calls=scheduler_config.is_async_mesos_calls())
        from dcos_commons_amd.mesos.local_master import LocalSchedulerDriver, local_master_from_env

        return LocalSchedulerDriver(local_master_from_env(scheduler_config.env), scheduler, framework_info)


def check_principal_override(framework_info: P.FrameworkInfo, scheduler_config) -> None:
    """The credential's principal is always ``FrameworkInfo.principal`` (the master rejects a
    credential for another principal). ``SDK_MESOS_PRINCIPAL`` names the principal of hand-built
    drivers (``SchedulerConfig.mesos_credential``); set to a different value for the scheduler it
    would be silently ignored, so that is refused as a configuration error instead."""
    override = scheduler_config.env.get_optional("SDK_MESOS_PRINCIPAL", "")
    if override and override != framework_info.principal:
        raise ValueError(f"SDK_MESOS_PRINCIPAL={override!r} differs from the framework principal "
                         f"{framework_info.principal!r}; the scheduler authenticates as the framework principal "
                         f"(set FRAMEWORK_PRINCIPAL / service.principal instead)")


def default_driver_factory(scheduler_config) -> Callable:
    """``driver_factory(scheduler, framework_info)`` for FrameworkRunner."""
    factory = SchedulerDriverFactory()
    master = scheduler_config.mesos_master_url()
    secret = scheduler_config.env.get_optional("SDK_MESOS_SECRET", "")

    def create(sched, info):
        check_principal_override(info, scheduler_config)
        return factory.create(sched, info, master, scheduler_config, secret.encode("utf-8") if secret else None)

    return create
