"""The C++ service CLI against the reference Go CLI's own fixtures.

The reference CLI tests (cli/queries/plan_test.go, pod_test.go) feed canned scheduler responses
(cli/queries/testdata/responses/scheduler/*) through an httptest server and compare the printed
output. Here the same fixtures are read in place: the ``inputJSON``/``expectedOutput`` pairs of every
``TestStatusTree*`` case are extracted from the Go sources, served by a local HTTP server, and
``sdk-cli`` must print exactly the expected tree; the plan-command cases check the success,
not-found and already-reported messages. Skipped when the reference tree is absent.
"""
import http.server
import json
import os
import re
import subprocess
import threading

import pytest

from conftest import reference_path

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "native", "build", "sdk-cli")
QUERIES = reference_path("cli", "queries")

pytestmark = pytest.mark.skipif(QUERIES is None or not os.path.exists(CLI),
                                reason="reference CLI fixtures or sdk-cli binary absent")


def _go_cases(filename, func_prefix):
    """(test name, input JSON, expected output, helper call) for every Go test case whose name
    starts with ``func_prefix``; raw-string (`...`) and quoted literals are both understood."""
    src = open(os.path.join(QUERIES, filename), encoding="utf-8").read()
    out = []
    for m in re.finditer(r"func \(suite \*\w+\) (" + func_prefix + r"\w*)\(\) \{(.*?)\n\}\n", src, re.S):
        name, body = m.group(1), m.group(2)

        def lit(var):
            mm = re.search(var + r" := `(.*?)`", body, re.S)
            if mm:
                return mm.group(1)
            mm = re.search(var + r' := "((?:[^"\\]|\\.)*)"', body)
            return json.loads('"' + mm.group(1) + '"') if mm else None
        inp = lit("inputJSON")
        if inp is None:
            mm = re.search(r'\[\]byte\("((?:[^"\\]|\\.)*)"\)', body)
            inp = json.loads('"' + mm.group(1) + '"') if mm else None
        call = re.search(r"result, err := (\w+)\(", body)
        out.append((name, inp, lit("expectedOutput"), call.group(1) if call else None))
    return out


class _Canned(http.server.BaseHTTPRequestHandler):
    routes = {}

    def log_message(self, *a):
        pass

    def _reply(self):
        status, body, ctype = self.routes.get((self.command, self.path.split("?")[0]), (404, b"", "text/plain"))
        self.server.requests.append((self.command, self.path))
        self.send_response(status)
        self.send_header("Content-Type", ctype)
        self.send_header("Content-Length", str(len(body)))
        self.end_headers()
        self.wfile.write(body)

    do_GET = do_POST = do_PUT = _reply


@pytest.fixture
def canned():
    class Handler(_Canned):
        routes = {}
    srv = http.server.ThreadingHTTPServer(("127.0.0.1", 0), Handler)
    srv.requests = []
    t = threading.Thread(target=srv.serve_forever, daemon=True)
    t.start()

    def route(method, path, status, body, ctype="application/json"):
        Handler.routes[(method, path)] = (status, body if isinstance(body, bytes) else body.encode(), ctype)

    def cli(*args):
        r = subprocess.run([CLI, "--url", f"http://127.0.0.1:{srv.server_address[1]}", *args],
                           capture_output=True, text=True, timeout=30)
        return r.returncode, r.stdout, r.stderr
    yield route, cli, srv
    srv.shutdown()


def _fixture(name):
    with open(os.path.join(QUERIES, "testdata", "responses", "scheduler", name), "rb") as f:
        return f.read()


PLAN_TREES = _go_cases("plan_test.go", "TestStatusTree") if QUERIES else []
POD_TREES = _go_cases("pod_test.go", "TestStatusTree") if QUERIES else []


@pytest.mark.parametrize("name,inp,expected,_", PLAN_TREES, ids=[c[0] for c in PLAN_TREES])
def test_plan_status_tree(canned, name, inp, expected, _):
    route, cli, _srv = canned
    route("GET", "/v1/plans/deploy", 200, inp)
    rc, out, err = cli("plan", "status", "deploy")
    assert rc == 0, err
    assert out.rstrip("\n") == expected


@pytest.mark.parametrize("name,inp,expected,helper", POD_TREES, ids=[c[0] for c in POD_TREES])
def test_pod_status_tree(canned, name, inp, expected, helper):
    route, cli, _srv = canned
    if helper == "toServiceTree":
        route("GET", "/v1/pod/status", 200, inp)
        rc, out, err = cli("pod", "status")
    else:
        pod = json.loads(inp)["name"]
        route("GET", f"/v1/pod/{pod}/status", 200, inp)
        rc, out, err = cli("pod", "status", pod)
    assert rc == 0, err
    assert out.rstrip("\n") == expected


def test_status_tree_cases_were_found():
    assert len(PLAN_TREES) >= 8 and len(POD_TREES) >= 5


def test_plan_status_raw_json_and_417(canned):
    route, cli, _srv = canned
    body = _fixture("plan-status.json")
    route("GET", "/v1/plans/deploy", 417, body)
    rc, out, _ = cli("plan", "status", "deploy")          # 417 (plan has errors) still renders
    assert rc == 0 and out.startswith("deploy (serial strategy) (")
    rc, out, _ = cli("--json", "plan", "status", "deploy")
    assert rc == 0 and json.loads(out) == json.loads(body)


@pytest.mark.parametrize("args,endpoint,fixture,expected", [
    (["force-complete", "deploy", "hello", "hello-0:[server]"], "/v1/plans/deploy/forceComplete", "force-complete.json",
     '"deploy" plan: step "hello-0:[server]" in phase "hello" has been forced to complete.'),
    (["force-restart", "deploy", "hello", "hello-0:[server]"], "/v1/plans/deploy/restart", "restart.json",
     '"deploy" plan: step "hello-0:[server]" in phase "hello" has been restarted.'),
    (["force-restart", "deploy", "hello"], "/v1/plans/deploy/restart", "restart.json",
     '"deploy" plan: phase "hello" has been restarted.'),
    (["force-restart", "deploy"], "/v1/plans/deploy/restart", "restart.json", '"deploy" plan has been restarted.'),
    (["pause", "deploy", "hello"], "/v1/plans/deploy/interrupt", "interrupt.json",
     '"deploy" plan: phase "hello" has been paused.'),
    (["pause", "deploy"], "/v1/plans/deploy/interrupt", "interrupt.json", '"deploy" plan has been paused.'),
    (["resume", "deploy", "hello"], "/v1/plans/deploy/continue", "continue.json",
     '"deploy" plan: phase "hello" has been resumed.'),
    (["resume", "deploy"], "/v1/plans/deploy/continue", "continue.json", '"deploy" plan has been resumed.'),
])
def test_plan_commands(canned, args, endpoint, fixture, expected):
    route, cli, srv = canned
    route("POST", endpoint, 200, _fixture(fixture))
    rc, out, err = cli("plan", *args)
    assert rc == 0, err
    assert out == expected + "\n"
    method, path = srv.requests[-1]
    assert method == "POST" and path.startswith(endpoint)
    if len(args) > 2:
        assert "phase=" + args[2] in path


def test_plan_command_invalid_response_could_not(canned):
    route, cli, _srv = canned
    route("POST", "/v1/plans/deploy/interrupt", 200, '{"not-a-valid-key":"Nope!"}')
    rc, out, _ = cli("plan", "pause", "deploy", "hello")
    assert rc == 0 and out == '"deploy" plan: phase "hello" could not be paused.\n'


@pytest.mark.parametrize("cmd", [["pause", "bad-name"], ["pause", "deploy", "bad-phase"], ["resume", "bad-name"],
                                 ["resume", "deploy", "bad-phase"]])
def test_plan_command_not_found(canned, cmd):
    route, cli, _srv = canned
    nf = _fixture("not-found.txt")
    for ep in ("interrupt", "continue"):
        route("POST", f"/v1/plans/{cmd[1]}/{ep}", 404, nf, "text/plain")
    rc, out, err = cli("plan", *cmd)
    assert rc != 0 and err.strip() == "Plan, phase, and/or step does not exist"


@pytest.mark.parametrize("cmd", [["pause", "deploy", "hello"], ["resume", "deploy", "hello"]])
def test_plan_command_already_reported(canned, cmd):
    route, cli, _srv = canned
    ar = _fixture("already-reported.txt")
    route("POST", "/v1/plans/deploy/interrupt", 208, ar, "text/plain")
    route("POST", "/v1/plans/deploy/continue", 208, ar, "text/plain")
    rc, out, err = cli("plan", *cmd)
    assert rc != 0
    assert err.strip() == "Cannot execute command. Command has already been issued or the plan has completed"


def test_plan_list_fixture(canned):
    route, cli, _srv = canned
    route("GET", "/v1/plans", 200, _fixture("plans.json"))
    rc, out, _ = cli("plan", "list")
    assert rc == 0 and json.loads(out) == json.loads(_fixture("plans.json"))


def test_plan_start_parameters(canned):
    route, cli, srv = canned
    route("POST", "/v1/plans/sidecar/start", 200, '{"message": "Received cmd: start"}')
    rc, out, _ = cli("plan", "start", "sidecar", "-p", "var=value", "-p", "var4=value=more")
    assert rc == 0 and json.loads(out)["message"] == "Received cmd: start"
