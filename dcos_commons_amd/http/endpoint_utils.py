"""DNS/VIP naming helpers (reference sdk/.../http/EndpointUtils.java)."""
from __future__ import annotations

SERVICE_ARTIFACT_URI_FORMAT = "http://%s/v1/artifacts/template/%s/%s/%s/%s"


def to_endpoint(hostname: str, port: int) -> str:
    return f"{hostname}:{port}"


def remove_slashes(name: str) -> str:
    return name.replace("/", "")


def replace_dots_with_dashes(name: str) -> str:
    return name.replace(".", "-")


def _reverse_slashed_segments_with_dashes(name: str) -> str:
    return "-".join(reversed([s for s in name.split("/") if s]))


def to_auto_ip_domain(service_name: str, scheduler_config) -> str:
    return f"{remove_slashes(replace_dots_with_dashes(service_name))}.{scheduler_config.autoip_tld()}"


def to_auto_ip_hostname(service_name: str, task_name: str, scheduler_config) -> str:
    return (f"{_reverse_slashed_segments_with_dashes(replace_dots_with_dashes(task_name))}."
            f"{to_auto_ip_domain(service_name, scheduler_config)}")


def to_auto_ip_endpoint(service_name: str, task_name: str, port: int, scheduler_config) -> str:
    return to_endpoint(to_auto_ip_hostname(service_name, task_name, scheduler_config), port)


def to_scheduler_auto_ip_hostname(service_name: str, scheduler_config) -> str:
    return to_auto_ip_hostname(scheduler_config.marathon_name(), service_name, scheduler_config)


def to_scheduler_auto_ip_endpoint(service_name: str, scheduler_config) -> str:
    return to_auto_ip_endpoint(scheduler_config.marathon_name(), service_name, scheduler_config.api_server_port(),
                               scheduler_config)


def to_vip_domain(service_name: str, scheduler_config) -> str:
    return f"{remove_slashes(service_name)}.{scheduler_config.vip_tld()}"


def to_vip_hostname(service_name: str, scheduler_config, vip_name: str) -> str:
    return f"{remove_slashes(vip_name)}.{to_vip_domain(service_name, scheduler_config)}"


def to_vip_endpoint(service_name: str, scheduler_config, vip_name: str, vip_port: int) -> str:
    return to_endpoint(to_vip_hostname(service_name, scheduler_config, vip_name), vip_port)


def template_url_factory(service_name: str, scheduler_config, prefix: str = ""):
    """ArtifactResource.getUrlFactory: task config templates are served by the scheduler. With a
    ``prefix`` (the service's name in a multi-service scheduler) the URL goes through
    ``/v1/service/<sanitized prefix>``, slashes becoming dots (MultiArtifactResource.getUrlFactory)."""
    from dcos_commons_amd.offer.common_id_utils import to_sanitized_service_name

    host_port = to_scheduler_auto_ip_endpoint(service_name, scheduler_config)
    prefix = to_sanitized_service_name(prefix) if prefix else ""

    def factory(config_id, pod_type: str, task_name: str, config_name: str) -> str:
        if prefix:
            return (f"http://{host_port}/v1/service/{prefix}/artifacts/template/"
                    f"{config_id}/{pod_type}/{task_name}/{config_name}")
        return SERVICE_ARTIFACT_URI_FORMAT % (host_port, config_id, pod_type, task_name, config_name)

    return factory
