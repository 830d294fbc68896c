"""YAML ServiceSpec parsing/validation and the mustache renderer.

Fixtures: the reference's own spec fixtures (sdk/scheduler/src/test/resources/*.yml) are read in
place when the reference tree is present (reference: specification/DefaultServiceSpecTest,
yaml/RawServiceSpecTest, yaml/TemplateUtilsTest)."""
import glob
import os

import pytest

from conftest import reference_path
from dcos_commons_amd.scheduler.scheduler_config import SchedulerConfig
from dcos_commons_amd.specification import specs as S
from dcos_commons_amd.specification.yaml import mappers
from dcos_commons_amd.specification.yaml import template_utils as TU
from dcos_commons_amd.specification.yaml.raw import RawServiceSpec

FIXTURES = reference_path("sdk", "scheduler", "src", "test", "resources")
CFG = SchedulerConfig.for_testing()
needs_fixtures = pytest.mark.skipif(FIXTURES is None, reason="reference fixtures not present")


class _Reader:
    def read(self, path):
        return f"template for {path}"


def build(path, env=None, reader=True):
    raw = RawServiceSpec.new_builder(path).set_env(env or {}).build()
    g = mappers.ServiceSpecGenerator(raw, CFG, os.path.dirname(path), env or {})
    if reader:
        g.reader = _Reader()
    return raw, g.build()


def fixture_files(prefix):
    if FIXTURES is None:
        return []
    return sorted(os.path.basename(p) for p in glob.glob(os.path.join(FIXTURES, prefix + "*.yml")))


VALID_EXCEPTIONS = {"valid-finished.yml"}  # uses the retired FINISHED goal: must be rejected
INVALID_BUILD_OK = {"invalid-config-file.yml", "invalid-plan-steps.yml"}  # fail later (reader / plans)


@needs_fixtures
@pytest.mark.parametrize("name", [n for n in fixture_files("valid-") if n not in VALID_EXCEPTIONS])
def test_valid_fixture_parses_and_round_trips(name):
    _, spec = build(os.path.join(FIXTURES, name))
    again = S.ServiceSpec.from_json_bytes(spec.to_json_bytes())
    assert again == spec
    assert S.loopback_check(spec) is not None


@needs_fixtures
@pytest.mark.parametrize("name", [n for n in fixture_files("invalid-") if n not in INVALID_BUILD_OK])
def test_invalid_fixture_rejected(name):
    with pytest.raises(Exception):
        build(os.path.join(FIXTURES, name))


@needs_fixtures
def test_invalid_config_file_missing_template():
    with pytest.raises((FileNotFoundError, OSError, Exception)):
        build(os.path.join(FIXTURES, "invalid-config-file.yml"), reader=False)


@needs_fixtures
def test_invalid_plan_steps_fail_at_scheduler_build():
    from dcos_commons_amd.scheduler.scheduler_builder import SchedulerBuilder
    from dcos_commons_amd.storage.mem_persister import MemPersister

    raw, spec = build(os.path.join(FIXTURES, "invalid-plan-steps.yml"))
    with pytest.raises(Exception):
        SchedulerBuilder(spec, CFG, MemPersister()).set_plans_from(raw).build()


@needs_fixtures
def test_goal_finished_rejected_with_reference_message():
    with pytest.raises(Exception) as e:
        build(os.path.join(FIXTURES, "valid-finished.yml"))
    assert "Unsupported GoalState FINISHED in task meta-data-task, expected one of" in str(e.value)


@needs_fixtures
def test_port_ranges_defaults():
    _, spec = build(os.path.join(FIXTURES, "ranges.yml"))
    ports = [r for r in spec.pods[0].tasks[0].resource_set.resources if r.name == "ports"]
    assert len(ports) == 2
    assert ports[0].port_name == "name1" and ports[0].env_key == "key1"
    assert [(r.begin, r.end) for r in ports[0].ranges] == [(1, 21), (2000, 5050)]
    assert [(r.begin, r.end) for r in ports[1].ranges] == [(0, 21), (5000, 65535)]


@needs_fixtures
def test_gpu_resource_fixture():
    _, spec = build(os.path.join(FIXTURES, "valid-gpu-resource.yml"))
    assert spec.uses_gpus()
    from dcos_commons_amd.config.validate import service_requests_gpu_resources

    assert service_requests_gpu_resources(spec)


@needs_fixtures
def test_duplicate_keys_are_an_error():
    with pytest.raises(Exception) as e:
        build(os.path.join(FIXTURES, "invalid-duplicate-count.yml"))
    assert "Duplicate field 'count'" in str(e.value)


# -- mustache ---------------------------------------------------------------------------------

def test_mustache_basic_and_escape():
    assert TU.render_mustache("t", "a={{A}} b={{{B}}}", {"A": "<x>", "B": "<y>"}, []) == "a=&lt;x&gt; b=<y>"
    assert TU.render_mustache("t", "{{A}}", {"A": "&\"'`="}, []) == "&amp;&quot;&#39;&#x60;&#x3D;"


def test_mustache_sections_and_inverted():
    tpl = "{{#FLAG}}on{{/FLAG}}{{^FLAG}}off{{/FLAG}}"
    assert TU.render_mustache("t", tpl, {"FLAG": "true"}, []) == "on"
    assert TU.render_mustache("t", tpl, {"FLAG": "false"}, []) == "off"
    assert TU.render_mustache("t", tpl, {}, []) == "off"


def test_mustache_missing_values_reported_with_lines():
    missing = []
    out = TU.render_mustache("t", "x\n{{A}}\n{{B}}", {"A": "1"}, missing)
    assert out == "x\n1\n"
    assert [(m.name, m.line) for m in missing] == [("B", 3)]
    with pytest.raises(TU.MustacheError):
        TU.render_mustache_throw_if_missing("t", "{{NOPE}}", {})


@needs_fixtures
def test_render_reference_template_fixture():
    path = os.path.join(FIXTURES, "test-render.yml")
    content = open(path).read()
    missing = []
    TU.render_mustache("test-render.yml", content, {}, missing)
    assert missing  # the fixture is all template variables
    names = {m.name for m in missing}
    env = {n: "1" for n in names}
    assert TU.render_mustache("test-render.yml", content, env, []) is not None


# -- helloworld specs in this repo --------------------------------------------------------------

def test_helloworld_gpu_spec_requests_gpus():
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {"FRAMEWORK_NAME": "hw", "FRAMEWORK_PRINCIPAL": "p", "FRAMEWORK_USER": "nobody", "HELLO_COUNT": "8",
           "HELLO_PLACEMENT": '[["hostname", "UNIQUE"]]', "HELLO_CPUS": "0.1", "HELLO_GPUS": "1", "HELLO_MEM": "252",
           "HELLO_DISK": "25", "SLEEP_DURATION": "1000", "GPU_PROBE_CMD": "amd-gpu-probe --readiness"}
    raw, spec = build(os.path.join(root, "frameworks", "helloworld", "specs", "gpu.yml"), env)
    assert spec.uses_gpus() and spec.pods[0].count == 8
    assert raw.plans["deploy"]["strategy"] == "parallel"
    t = spec.pods[0].tasks[0]
    assert t.readiness_check.command == "amd-gpu-probe --readiness"


def test_loopback_parse_cache_is_thread_safe():
    """The loopback parse cache is shared by every service of a multi-service scheduler; concurrent
    checks that evict entries must neither raise nor return another spec's parse."""
    from concurrent.futures import ThreadPoolExecutor
    from dataclasses import replace

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {"FRAMEWORK_NAME": "hw", "FRAMEWORK_PRINCIPAL": "p", "FRAMEWORK_USER": "nobody", "HELLO_COUNT": "2",
           "HELLO_PLACEMENT": '[["hostname", "UNIQUE"]]', "HELLO_CPUS": "0.1", "HELLO_GPUS": "1", "HELLO_MEM": "252",
           "HELLO_DISK": "25", "SLEEP_DURATION": "1000", "GPU_PROBE_CMD": "amd-gpu-probe --readiness"}
    _, base = build(os.path.join(root, "frameworks", "helloworld", "specs", "gpu.yml"), env)
    specs = [replace(base, name=f"svc-{i}") for i in range(80)]       # more than the cache holds

    def check(i):
        s = specs[i % len(specs)]
        assert S._parse_cached(s.to_json_bytes()) == s
        return S.loopback_check(s) is not None

    with ThreadPoolExecutor(8) as pool:
        assert all(pool.map(check, range(800)))
