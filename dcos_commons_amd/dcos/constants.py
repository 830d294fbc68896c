"""DC/OS cluster constants (reference sdk/.../dcos/DcosConstants.java)."""

MESOS_MASTER = "master.mesos"
MESOS_MASTER_URI = "http://" + MESOS_MASTER
DEFAULT_SECRET_STORE_URI = MESOS_MASTER_URI + "/secrets/v1/secret/default/"
CA_BASE_URI = MESOS_MASTER_URI + "/ca/api/v2/"
IAM_AUTH_URL = MESOS_MASTER_URI + "/acs/api/v1/auth/login"
DEFAULT_GPU_POLICY = False
DEFAULT_IP_PROTOCOL = "tcp"
OVERLAY_DYNAMIC_PORT_RANGE_START = 1025
OVERLAY_DYNAMIC_PORT_RANGE_END = 2025
DEFAULT_SERVICE_USER = "root"
MESOS_MASTER_ZK_CONNECTION_STRING = MESOS_MASTER + ":2181"
MESOS_LEADER = "leader.mesos"
MESOS_LEADER_URI = "http://" + MESOS_LEADER
DEFAULT_OVERLAY_NETWORK = "dcos"
DEFAULT_BRIDGE_NETWORK = "mesos-bridge"
SUPPORTED_OVERLAY_NETWORKS = frozenset([DEFAULT_OVERLAY_NETWORK, DEFAULT_BRIDGE_NETWORK])


def network_supports_port_mapping(network_name: str) -> bool:
    return network_name == DEFAULT_BRIDGE_NETWORK


def is_supported_network(network_name: str) -> bool:
    return network_name in SUPPORTED_OVERLAY_NETWORKS
