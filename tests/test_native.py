"""Native tools: C++ unit tests, sdk-bootstrap template rendering, sdk-cli against a live scheduler
API, and (on the GPU box) the standalone amd-gpu-probe. Reference: sdk/bootstrap/main_test.go,
cli/queries/*_test.go."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, "native", "build")


# Every native test runs against the release build and against an AddressSanitizer + UBSan build
# of the same sources (the reference has no native code, so no sanitizers; the C++
# natives here get them). Sanitizer findings abort the tool, which fails the test.
SANITIZER_ENV = {"ASAN_OPTIONS": "halt_on_error=1:abort_on_error=1:detect_leaks=1",
                 "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1"}


@pytest.fixture(scope="module", params=["release", "sanitize"])
def tools(request):
    sys.path.insert(0, ROOT)
    from dcos_commons_amd.ops import build

    sanitize = request.param == "sanitize"
    try:
        targets = build.build_cpp_tools(sanitize=sanitize)
    except Exception as e:  # noqa: BLE001
        pytest.skip(f"native toolchain unavailable: {e}")
    saved = {k: os.environ.get(k) for k in SANITIZER_ENV}
    if sanitize:
        os.environ.update(SANITIZER_ENV)
    yield {os.path.basename(t): t for t in targets}
    for k, v in saved.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v


def test_native_unit_tests(tools):
    r = subprocess.run([tools["native-tests"]], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr


def test_tls_library_round_trips(tools):
    """Keys, CSRs, root/intermediate CAs, chain checks, PKCS#12 stores, RS256/JWT and error paths
    of the TLS crypto code (native/tests/test_tls.cpp), instrumented in the sanitizer build."""
    r = subprocess.run([tools["tls-tests"]], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "tls tests passed" in r.stdout, r.stdout + r.stderr


def test_bootstrap_renders_config_templates(tools, tmp_path):
    sandbox = tmp_path
    (sandbox / "tpl.conf").write_text("name={{NAME}}\n{{#FLAG}}flag on\n{{/FLAG}}{{^OFF}}off is off\n{{/OFF}}"
                                      "raw={{{RAW}}} esc={{RAW}}\n")
    out = sandbox / "out.conf"
    env = dict(os.environ, MESOS_SANDBOX=str(sandbox), NAME="node-0", FLAG="true", OFF="false", RAW="<a&b>",
               CONFIG_TEMPLATE_MAIN=f"tpl.conf,{out}", SECRET_TOKEN="hunter2")
    r = subprocess.run([tools["sdk-bootstrap"], "-resolve=false", "-install-certs=false"], env=env,
                       capture_output=True, text=True, timeout=30)
    assert r.returncode == 0, r.stderr
    assert out.read_text() == "name=node-0\nflag on\noff is off\nraw=<a&b> esc=&lt;a&amp;b&gt;\n"
    # credentials are masked when the environment is printed
    assert "SECRET_TOKEN=********" in r.stderr and "hunter2" not in r.stderr
    assert "SDK Bootstrap successful." in r.stderr


def test_bootstrap_template_errors(tools, tmp_path):
    env = dict(os.environ, MESOS_SANDBOX=str(tmp_path), CONFIG_TEMPLATE_X="missing.conf,/dev/null")
    r = subprocess.run([tools["sdk-bootstrap"], "-resolve=false", "-install-certs=false"], env=env,
                       capture_output=True, text=True, timeout=30)
    assert r.returncode != 0 and "doesn't exist" in r.stderr
    (tmp_path / "big").write_text("x" * 100)
    env = dict(os.environ, MESOS_SANDBOX=str(tmp_path), CONFIG_TEMPLATE_X="big,/dev/null")
    r = subprocess.run([tools["sdk-bootstrap"], "-resolve=false", "-install-certs=false", "-template-max-bytes=10"],
                       env=env, capture_output=True, text=True, timeout=30)
    assert r.returncode != 0 and "exceeds maximum" in r.stderr


def test_bootstrap_resolution_and_task_ip(tools):
    env = dict(os.environ, TASK_NAME="localhost", FRAMEWORK_HOST="", LIBPROCESS_IP="10.1.2.3")
    r = subprocess.run([tools["sdk-bootstrap"], "-get-task-ip"], env=env, capture_output=True, text=True, timeout=30)
    assert r.returncode == 0 and r.stdout == "10.1.2.3"
    r = subprocess.run([tools["sdk-bootstrap"], "-resolve-hosts=localhost", "-self-resolve=false",
                        "-install-certs=false", "-template=false", "-resolve-timeout=10s"],
                       env=env, capture_output=True, text=True, timeout=30)
    assert r.returncode == 0 and "Resolved 'localhost'" in r.stderr
    r = subprocess.run([tools["sdk-bootstrap"], "-resolve-hosts=no-such-host.invalid", "-self-resolve=false",
                        "-resolve-timeout=1s", "-install-certs=false"], env=env, capture_output=True, text=True,
                       timeout=30)
    assert r.returncode != 0 and "Time ran out" in r.stderr


def test_bootstrap_gpu_check_rejects_missing_device(tools):
    env = dict(os.environ, HIP_VISIBLE_DEVICES="63")
    r = subprocess.run([tools["sdk-bootstrap"], "-resolve=false", "-install-certs=false", "-template=false"],
                       env=env, capture_output=True, text=True, timeout=30)
    assert r.returncode != 0  # no KFD here, or no GPU 63 on the box
    r = subprocess.run([tools["sdk-bootstrap"], "-resolve=false", "-install-certs=false", "-template=false",
                        "-gpu-check=false"], env=env, capture_output=True, text=True, timeout=30)
    assert r.returncode == 0


def test_cli_against_live_scheduler(tools):
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from test_e2e_helloworld import Cluster

    with Cluster() as c:
        c.wait_plan("deploy")
        url = f"http://127.0.0.1:{c.runner.framework_runner.api_server.port}"

        def cli(*args):
            r = subprocess.run([tools["sdk-cli"], "--url", url, *args], capture_output=True, text=True, timeout=30)
            return r.returncode, r.stdout, r.stderr

        rc, out, _ = cli("plan", "status", "deploy")
        assert rc == 0
        lines = out.splitlines()
        assert lines[0] == "deploy (serial strategy) (COMPLETE)"
        assert lines[1] == "├─ hello (serial strategy) (COMPLETE)"
        assert "│  └─ hello-1:[server] (COMPLETE)" in lines
        assert lines[-1] == "   └─ world-1:[server] (COMPLETE)"
        rc, out, _ = cli("plan", "list")
        assert rc == 0 and '"deploy"' in out and '"recovery"' in out
        rc, out, _ = cli("pod", "status")
        assert rc == 0 and out.splitlines()[0] == "hello-world" and "hello-0-server (RUNNING)" in out
        rc, out, _ = cli("pod", "status", "world-1")
        assert rc == 0 and out.splitlines() == ["world-1", "└─ world-1-server (RUNNING)"]
        rc, _, err = cli("plan", "pause", "deploy")
        assert rc == 1 and "Command has already been issued or the plan has completed" in err
        rc, _, err = cli("plan", "resume", "deploy", "nope")
        assert rc == 1 and err.strip() == "Plan, phase, and/or step does not exist"
        rc, _, err = cli("pod", "info", "nope-9")
        assert rc == 2 and "404" in err
        rc, out, _ = cli("debug", "state", "framework_id")
        assert rc == 0 and "fw-" in out
        rc, out, _ = cli("describe")
        assert rc == 0 and '"name": "hello-world"' in out
        rc, out, _ = cli("health")
        assert rc == 0 and '"value": 200' in out
        rc, out, _ = cli("pod", "restart", "hello-0")
        assert rc == 0 and '"pod": "hello-0"' in out


@pytest.mark.gpu
def test_amd_gpu_probe_binary():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    sys.path.insert(0, ROOT)
    from dcos_commons_amd.ops import build

    exe = build.build_probe_binary()
    r = subprocess.run([exe, "--readiness", "--json"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    import json

    rep = json.loads(r.stdout)
    assert rep["healthy"] and rep["mem_bad_words"] == 0 and rep["gemm_rel_err"] < 1e-5
    r = subprocess.run([exe, "--full", "--json"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    rep = json.loads(r.stdout)
    assert rep["mfma_tflops"] > 500 and rep["hbm_copy_gbps"] > 2000


def test_cli_hdfs_plugin_argument_split(tools):
    """frameworks/hdfs/cli: everything after a leading `hdfs` section goes to bin/hdfs (main_test.go)."""
    env = dict(os.environ, SDK_CLI_DRY_RUN="1")

    def run(*args):
        r = subprocess.run([tools["sdk-cli"], *args], capture_output=True, text=True, timeout=30, env=env)
        return r.returncode, r.stdout.strip().split("\x1f")

    rc, cmd = run("hdfs", "dfs", "-ls", "/")
    assert rc == 0 and cmd[:6] == ["dcos", "task", "exec", "name-0-node", "bash", "-c"]
    assert cmd[6].endswith("bin/hdfs dfs -ls /")
    rc, cmd = run("--service", "hdfs", "--json", "hdfs", "dfsadmin", "-report", "--help")
    assert rc == 0 and cmd[6].endswith("bin/hdfs dfsadmin -report --help")  # plugin flags are not parsed
    r = subprocess.run([tools["sdk-cli"], "--url", "http://127.0.0.1:9", "plan", "hdfs"], capture_output=True,
                       text=True, timeout=30, env=env)
    assert "dcos" not in r.stdout  # `hdfs` is not the first argument: regular SDK section
