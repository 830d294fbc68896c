"""SDK-wide constants (reference sdk/.../offer/Constants.java:22-108)."""
from dcos_commons_amd.mesos import protos as P

DEPLOY_PLAN_NAME = "deploy"
RECOVERY_PLAN_NAME = "recovery"
UPDATE_PLAN_NAME = "update"
DECOMMISSION_PLAN_NAME = "decommission"

PORTS_RESOURCE_TYPE = "ports"
DISK_RESOURCE_TYPE = "disk"
CPUS_RESOURCE_TYPE = "cpus"
MEMORY_RESOURCE_TYPE = "mem"
GPUS_RESOURCE_TYPE = "gpus"
ANY_ROLE = "*"

DISPLAYED_PORT_VISIBILITY = P.DiscoveryInfo.EXTERNAL
OMITTED_PORT_VISIBILITY = P.DiscoveryInfo.CLUSTER
DEFAULT_TASK_DISCOVERY_VISIBILITY = P.DiscoveryInfo.CLUSTER

LONG_DECLINE_SECONDS = 3600
SHORT_DECLINE_SECONDS = 5
