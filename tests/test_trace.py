"""Chrome-trace spans (the reference has only the ``offers.process`` timer,
OfferProcessor.java:327-337; this SDK adds per-cycle / per-step / per-persister-op spans)."""
import json

import pytest

from dcos_commons_amd import trace
from dcos_commons_amd.mesos import protos as P
from dcos_commons_amd.storage.mem_persister import MemPersister

from test_e2e_helloworld import Cluster


@pytest.fixture
def tracing():
    was = trace.enabled()
    trace.TRACER.clear()
    trace.enable()
    yield trace.TRACER
    trace.TRACER.clear()
    if not was:
        trace.disable()


def test_disabled_span_is_shared_noop():
    was = trace.enabled()
    trace.disable()
    try:
        a, b = trace.span("x"), trace.span("y", k=1)
        assert a is b
        with a as s:
            s.set(n=1)
        assert not [e for e in trace.TRACER.events() if e["name"] in ("x", "y")]
    finally:
        if was:
            trace.enable()


def test_span_records_complete_event_and_error(tracing):
    with trace.span("work", "unit", n=3) as s:
        s.set(out=7)
    with pytest.raises(ValueError):
        with trace.span("boom"):
            raise ValueError("x")
    evs = {e["name"]: e for e in tracing.events()}
    assert evs["work"]["ph"] == "X" and evs["work"]["dur"] >= 0
    args = dict(evs["work"]["args"])
    assert args.pop("cpu_us") >= 0          # the thread's own CPU time inside the span
    assert args == {"n": 3, "out": 7}
    assert evs["boom"]["args"]["error"] == "ValueError"
    summary = tracing.summary()
    assert summary["work"]["count"] == 1 and summary["work"]["mean_ms"] >= 0


def test_ring_is_bounded():
    t = trace.Tracer(enabled=True, max_events=4)
    for i in range(10):
        with t.span(f"s{i}"):
            pass
    names = [e["name"] for e in t.events()]
    assert names == ["s6", "s7", "s8", "s9"] and t.dropped == 6


def test_tracing_persister_forwards(tracing, tmp_path):
    p = trace.TracingPersister(MemPersister())
    p.set_many({"/a/b": b"1", "/a/c": b"22"})
    assert p.get("/a/b") == b"1"
    assert sorted(p.get_children("/a")) == ["b", "c"]
    p.recursive_delete("/a")
    names = [e["name"] for e in tracing.events()]
    assert names == ["persister.set_many", "persister.get", "persister.get_children", "persister.recursive_delete"]
    assert {k: v for k, v in tracing.events()[0]["args"].items() if k != "cpu_us"} == {"n": 2, "bytes": 3}
    path = tracing.dump(str(tmp_path / "t.json"))
    doc = json.load(open(path))
    assert any(e.get("ph") == "M" for e in doc["traceEvents"])


def test_live_deploy_emits_cycle_evaluate_status_accept_spans(tracing):
    with Cluster(agents=4) as c:
        c.wait_plan("deploy")
        r = c.api.get("/v1/debug/trace?summary=true")
        assert r.status == 200
        spans = r.body["spans"]
        for name in ("offer_cycle", "evaluate", "status", "accept"):
            assert spans.get(name, {}).get("count", 0) >= 1, (name, spans)
        # every pod instance step was evaluated at least once
        steps = {e["args"]["step"] for e in tracing.events() if e["name"] == "evaluate"}
        assert any(s.startswith("hello-0") for s in steps) and any(s.startswith("world-1") for s in steps)
        statuses = [e["args"]["state"] for e in tracing.events() if e["name"] == "status"]
        assert P.TaskState.Name(P.TASK_RUNNING) in statuses
        doc = c.api.get("/v1/debug/trace?clear=true").body
        assert doc["traceEvents"] and doc["otherData"]["enabled"]
        assert not [e for e in tracing.events() if e["name"] == "evaluate" and e["ts"] < 0]
