"""helloworld integration-test configuration (reference: frameworks/helloworld/tests/config.py)."""
from dcos_commons_amd.testing.sdk import sdk_marathon, sdk_tasks

PACKAGE_NAME = "hello-world"
SERVICE_NAME = PACKAGE_NAME
DEFAULT_TASK_COUNT = 3


def task_count(key_name, service_name=SERVICE_NAME):
    return int(sdk_marathon.get_config(service_name)["env"][key_name])


def hello_task_count(service_name=SERVICE_NAME):
    return task_count("HELLO_COUNT", service_name)


def world_task_count(service_name=SERVICE_NAME):
    return task_count("WORLD_COUNT", service_name)


def configured_task_count(service_name=SERVICE_NAME):
    return hello_task_count(service_name) + world_task_count(service_name)


def check_running(service_name=SERVICE_NAME):
    sdk_tasks.check_running(service_name, configured_task_count(service_name))


def bump_hello_cpus(service_name=SERVICE_NAME):
    return sdk_marathon.bump_cpu_count_config(service_name, "HELLO_CPUS")


def bump_world_cpus(service_name=SERVICE_NAME):
    return sdk_marathon.bump_cpu_count_config(service_name, "WORLD_CPUS")


def close_enough(a, b):
    return abs(a - b) < 1e-5
