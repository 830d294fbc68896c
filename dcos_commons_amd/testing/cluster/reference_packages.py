"""The reference's unchanged packages (``frameworks/{helloworld,cassandra,hdfs}``) on the local
DC/OS stand-in.

A reference package is its ``universe/`` directory (options, ``marathon.json.mustache``,
``resource.json``) plus the scheduler artifact its Marathon app fetches: ``<name>-scheduler.zip``,
which the reference's build assembles from the framework's ``src/main/dist`` files and a start
script ``bin/<framework>``. Here that artifact is staged the same way from the same files, with
a start script that runs this SDK's scheduler main for the framework, and registered in the
cluster's artifact store; the Marathon stand-in fetches it (with ``bootstrap.zip``, this tree's
native ``sdk-bootstrap``) into the scheduler's sandbox and runs the package's own ``cmd``
unchanged: ``... && ./bootstrap -resolve=false -template=false && ./cassandra-scheduler/bin/cassandra
./cassandra-scheduler/svc.yml``. The JRE and libmesos URIs it also fetches are not needed and
are skipped.

    cluster = LocalCluster(packages=reference_packages(root), ...).start()
    stage_scheduler_artifacts(cluster, root)
"""
from __future__ import annotations

import os
import shutil
import stat
from typing import Dict, Optional

# package name -> (framework directory, start script name, scheduler main module)
FRAMEWORKS = {
    "hello-world": ("helloworld", "helloworld", "dcos_commons_amd.models.helloworld"),
    "cassandra": ("cassandra", "cassandra", "dcos_commons_amd.models.cassandra"),
    "hdfs": ("hdfs", "hdfs", "dcos_commons_amd.models.hdfs"),
}


def reference_root() -> Optional[str]:
    """$SDK_REFERENCE_ROOT, the reference checkout, or the staged ``ref_inputs/`` copy."""
    here = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
    for root in (os.environ.get("SDK_REFERENCE_ROOT", ""), "/root/reference", os.path.join(here, "ref_inputs")):
        if root and os.path.isdir(os.path.join(root, "frameworks", "cassandra", "universe")):
            return root
    return None


def reference_packages(root: str) -> Dict[str, str]:
    """Package name -> the reference's universe directory, for the packages it ships."""
    out = {}
    for name, (fw, _, _) in FRAMEWORKS.items():
        udir = os.path.join(root, "frameworks", fw, "universe")
        if os.path.isfile(os.path.join(udir, "marathon.json.mustache")):
            out[name] = udir
    return out


def stage_scheduler_artifacts(cluster, root: str) -> Dict[str, str]:
    """Stages ``<package>-scheduler.zip`` for every reference package (as its extracted tree:
    ``<package>-scheduler/`` with the ``src/main/dist`` files and ``bin/<framework>``) and
    registers it in ``cluster``'s artifact store. Returns artifact name -> staged directory."""
    staged = {}
    for name, (fw, script, module) in FRAMEWORKS.items():
        dist = os.path.join(root, "frameworks", fw, "src", "main", "dist")
        if not os.path.isdir(dist):
            continue
        base = os.path.join(cluster.work_dir, "artifacts", f"{name}-scheduler-zip")
        top = os.path.join(base, f"{name}-scheduler")
        os.makedirs(os.path.join(top, "bin"), exist_ok=True)
        for entry in os.listdir(dist):
            src = os.path.join(dist, entry)
            if os.path.isfile(src):
                shutil.copy2(src, os.path.join(top, entry))
        launcher = os.path.join(top, "bin", script)
        with open(launcher, "w", encoding="utf-8") as f:
            f.write("#!/bin/bash\n"
                    f"# {name} scheduler start script: this SDK's scheduler main for the package's svc.yml\n"
                    f'exec python3 -m {module} "$@"\n')
        os.chmod(launcher, os.stat(launcher).st_mode | stat.S_IXUSR | stat.S_IXGRP | stat.S_IXOTH)
        artifact = f"{name}-scheduler.zip"
        cluster.register_artifact(artifact, base)
        staged[artifact] = base
    return staged
