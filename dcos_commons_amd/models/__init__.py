"""Framework schedulers built on the SDK: ``helloworld``, ``cassandra``, ``hdfs``."""
from __future__ import annotations

import os

FRAMEWORKS_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                              "frameworks")


def resolve_spec(path: str, framework: str) -> str:
    """A scheduler's spec argument: an existing path as given, else a file of the framework's
    bundled specs (``frameworks/<framework>/specs``, overridable with ``<FRAMEWORK>_SPEC_DIR``) --
    what the scheduler artifact unpacks next to the scheduler on DC/OS."""
    if os.path.exists(path):
        return path
    spec_dir = os.environ.get(f"{framework.upper()}_SPEC_DIR") or os.path.join(FRAMEWORKS_DIR, framework, "specs")
    return os.path.join(spec_dir, os.path.basename(path))
