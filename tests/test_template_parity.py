"""The task-side renderer (``sdk-bootstrap``, ``native/common/mustache.cpp``) and the scheduler's
renderer (``specification/yaml/template_utils.py``) produce the same bytes.

Tasks render their config templates with the native bootstrap; the scheduler renders the same
templates when it validates a spec and when the harness reads ``get_task_config``. A divergence
would mean the configuration a task runs with differs from the one the scheduler checked. For every
config template of every task launched by a deploy, the template is placed in a sandbox as the
task's URI fetch would place it, ``sdk-bootstrap`` renders it with exactly the launched TaskInfo's
environment (``CONFIG_TEMPLATE_*`` included), and the result must equal ``render_mustache`` of the
same template and environment, byte for byte.

Packages: this repository's cassandra and hdfs (always), and the reference's unchanged cassandra
and hdfs when its tree is present (their templates use sections, inverted sections, triple
mustaches and values the task environment lacks).
"""
import os
import subprocess

import pytest

from dcos_commons_amd.specification.yaml.template_utils import render_mustache

REF = os.environ.get("SDK_REFERENCE_ROOT", "/root/reference")
HAVE_REF = os.path.isdir(os.path.join(REF, "frameworks", "cassandra", "src", "main", "dist"))


@pytest.fixture(scope="module")
def bootstrap():
    from dcos_commons_amd.ops import build

    try:
        targets = build.build_cpp_tools()
    except Exception as e:  # noqa: BLE001
        pytest.skip(f"native toolchain unavailable: {e}")
    return [t for t in targets if t.endswith("sdk-bootstrap")][0]


def _deployed(which: str):
    """(service spec, launched TaskInfos) of a deploy of ``which``."""
    if which == "cassandra-repo":
        from test_cassandra import _deploy_ticks, runner
        res = runner().run(_deploy_ticks())
    elif which == "hdfs-repo":
        from test_hdfs import deploy_ticks, runner
        res = runner().run(deploy_ticks())
    elif which == "cassandra-reference":
        from test_cassandra import _deploy_ticks
        from test_reference_conformance import _cassandra_runner
        res = _cassandra_runner().run(_deploy_ticks())
    else:
        from test_hdfs import deploy_ticks
        from test_reference_conformance import _hdfs_runner
        res = _hdfs_runner().run(deploy_ticks())
    tasks = {}
    for a in res.sim.driver.accepts:
        for t in a.launched_tasks():
            tasks[t.name] = t
    return res.service_spec, list(tasks.values())


def _templates_of(spec, task_name: str):
    """config name -> template content for the task ``<pod>-<index>-<task>``."""
    for pod in spec.pods:
        prefix = pod.type + "-"
        if not task_name.startswith(prefix):
            continue
        rest = task_name[len(prefix):]
        idx, _, tname = rest.partition("-")
        if not idx.isdigit():
            continue
        for t in pod.tasks:
            if t.name == tname:
                return {c.name: c.template_content for c in t.config_files}
    return {}


PACKAGES = ["cassandra-repo", "hdfs-repo"] + (["cassandra-reference", "hdfs-reference"] if HAVE_REF else [])


@pytest.mark.parametrize("which", PACKAGES)
def test_bootstrap_and_scheduler_render_every_template_identically(which, bootstrap, tmp_path):
    from dcos_commons_amd.offer.evaluate.pod_info_builder import CONFIG_TEMPLATE_DOWNLOAD_PATH

    spec, tasks = _deployed(which)
    compared = 0
    for t in tasks:
        env = {v.name: v.value for v in t.command.environment.variables}
        # what the Mesos agent adds to every task (the bootstrap exports it as LIBPROCESS_IP too)
        env.update(MESOS_CONTAINER_IP="10.0.0.7", LIBPROCESS_IP="10.0.0.7")
        keys = sorted(k for k in env if k.startswith("CONFIG_TEMPLATE_"))
        if not keys:
            continue
        templates = _templates_of(spec, t.name)
        sandbox = tmp_path / t.name
        (sandbox / CONFIG_TEMPLATE_DOWNLOAD_PATH).mkdir(parents=True)
        expected = {}
        for k in keys:
            src, _, dst = env[k].partition(",")
            name = src[len(CONFIG_TEMPLATE_DOWNLOAD_PATH):]
            content = templates[name]
            (sandbox / src).write_text(content)
            expected[dst] = render_mustache(f"{t.name}:{name}", content, dict(env, MESOS_SANDBOX=str(sandbox)))
            os.makedirs(os.path.dirname(os.path.join(sandbox, dst)) or str(sandbox), exist_ok=True)
        run_env = dict(env, MESOS_SANDBOX=str(sandbox))
        r = subprocess.run([bootstrap, "-resolve=false", "-install-certs=false", "-self-resolve=false"],
                           env=run_env, cwd=str(sandbox), capture_output=True, text=True, timeout=60)
        assert r.returncode == 0, r.stderr[-2000:]
        for dst, want in expected.items():
            got = open(os.path.join(sandbox, dst), encoding="utf-8").read()
            assert got == want, f"{which} {t.name} {dst}: native and scheduler renderings differ"
            compared += 1
    # rendered files compared (3 cassandra nodes, 10 hdfs tasks, each with several templates)
    assert compared >= {"cassandra-repo": 6, "hdfs-repo": 26, "cassandra-reference": 14,
                        "hdfs-reference": 34}[which], compared
