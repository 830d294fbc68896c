"""``scheduler.launch_pipeline.LaunchPipeline``: streamed launches recorded behind the evaluation.

Every step's ACCEPT follows its durable record and the ACCEPTs keep step order; steps queued while
a write is in flight are recorded together; a failed record drops its steps' operations (reported
by ``drain``); ``drain`` returns only when everything submitted was recorded and sent. One writer
thread serves every cycle (parked in between) until ``close``. A ZooKeeper-backed DefaultScheduler turns it on by default
(``SDK_PIPELINE_LAUNCH_WRITES``); a local persister keeps the inline writes.
"""
import threading
import time

from dcos_commons_amd.scheduler.launch_pipeline import LaunchPipeline


def test_accepts_follow_their_record_in_order_and_coalesce():
    log = []
    gate = threading.Event()

    def record(recs):
        log.append(("record", list(recs)))
        gate.wait(5)                     # the first write is slow: later steps queue up behind it
        return True

    p = LaunchPipeline(record)
    p.submit(["a1", "a2"], lambda recs: log.append(("send", list(recs))))
    time.sleep(0.05)
    for step in ("b", "c", "d"):
        p.submit([step], lambda recs: log.append(("send", list(recs))))
    gate.set()
    assert p.drain() == []
    assert log == [("record", ["a1", "a2"]), ("send", ["a1", "a2"]),
                   ("record", ["b", "c", "d"]), ("send", ["b"]), ("send", ["c"]), ("send", ["d"])]
    assert p.writes == 2
    writer = p._thread
    p.close()
    # this pipeline's writer ended (other tests' schedulers may still own writers of that name)
    assert writer is not None and not writer.is_alive()


def test_failed_record_drops_the_operations():
    sent = []
    p = LaunchPipeline(lambda recs: "bad" not in recs)
    p.submit(["bad"], sent.append)
    assert p.drain() == [["bad"]] and sent == []
    p.submit(["ok"], sent.append)          # the next cycle reuses the parked writer
    assert p.drain() == [] and sent == [["ok"]]
    assert p.threads_started == 1
    p.close()


def test_one_writer_thread_serves_every_cycle_until_close():
    """a writer per cycle gave a sync-call v1 driver one new master connection per cycle."""
    seen = set()
    p = LaunchPipeline(lambda recs: seen.add(threading.get_ident()) or True, name="launch-writer-test")
    for cycle in range(20):
        p.submit([cycle], lambda recs: None)
        assert p.drain() == []
    assert p.threads_started == 1 and len(seen) == 1
    assert any(t.name == "launch-writer-test" for t in threading.enumerate())   # parked, not gone
    p.close()
    assert not any(t.name == "launch-writer-test" for t in threading.enumerate())


def test_record_exception_is_a_failed_record():
    def record(recs):
        raise RuntimeError("zk down")
    p = LaunchPipeline(record)
    p.submit(["x"], lambda recs: None)
    assert p.drain() == [["x"]]
    p.close()


def test_drain_without_submissions_returns_at_once():
    assert LaunchPipeline(lambda recs: True).drain() == []


def test_default_scheduler_pipelines_only_remote_persisters():
    from dcos_commons_amd.scheduler.default_scheduler import DefaultScheduler
    from dcos_commons_amd.scheduler.scheduler_config import SchedulerConfig
    from dcos_commons_amd.storage.mem_persister import MemPersister
    from dcos_commons_amd.storage.persister_cache import PersisterCache

    class Remote(MemPersister):
        remote = True

    def pipeline(persister, **env):
        s = DefaultScheduler.__new__(DefaultScheduler)
        s._pipeline = None
        s.scheduler_config = SchedulerConfig.for_testing(**env)
        s.state_store = type("S", (), {"persister": persister})()
        return s._launch_pipeline()

    assert pipeline(MemPersister()) is None
    assert isinstance(pipeline(PersisterCache(Remote())), LaunchPipeline)
    assert pipeline(PersisterCache(Remote()), SDK_PIPELINE_LAUNCH_WRITES="false") is None
    assert isinstance(pipeline(MemPersister(), SDK_PIPELINE_LAUNCH_WRITES="true"), LaunchPipeline)
