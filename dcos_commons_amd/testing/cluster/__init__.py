"""Local DC/OS stand-in for the system-integration tier (see ``cluster.py``)."""
from dcos_commons_amd.testing.cluster.cluster import LocalCluster, TaskView, current, use  # noqa: F401
from dcos_commons_amd.testing.cluster.marathon import LocalMarathon, scheduler_task_prefix  # noqa: F401
from dcos_commons_amd.testing.cluster.packages import LocalCosmos  # noqa: F401
