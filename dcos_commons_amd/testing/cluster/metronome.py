"""Metronome stand-in: one-off jobs of the local cluster (the reference's tests run data
read/write jobs through it, ``testing/sdk_jobs.py``).

A job definition is Metronome's JSON (``{"id", "run": {"cmd", "env", "maxLaunchDelay"?, ...}}``);
each run executes ``run.cmd`` under ``bash -c`` in its own sandbox with ``run.env`` plus the
cluster's task environment, and lands in the job's history as a successful or failed run.
"""
from __future__ import annotations

import copy
import os
import subprocess
import tempfile
import threading
import time
import uuid
from typing import Dict, List


class LocalMetronome:
    def __init__(self, cluster):
        self.cluster = cluster
        self._jobs: Dict[str, dict] = {}
        self._history: Dict[str, Dict[str, List[dict]]] = {}
        self._active: Dict[str, subprocess.Popen] = {}
        self._lock = threading.Lock()

    def add_job(self, job: dict) -> None:
        jid = job["id"]
        with self._lock:
            if jid in self._jobs:
                raise ValueError(f"Job with id {jid} already exists")
            self._jobs[jid] = copy.deepcopy(job)
            self._history[jid] = {"successfulFinishedRuns": [], "failedFinishedRuns": []}

    def remove_job(self, job_id: str, stop_current_runs: bool = True) -> None:
        with self._lock:
            if job_id not in self._jobs:
                raise KeyError(f"Job '{job_id}' does not exist")
            del self._jobs[job_id]
            procs = [p for rid, p in self._active.items() if rid.startswith(job_id + "/")]
        if stop_current_runs:
            for p in procs:
                p.kill()

    def job(self, job_id: str, embed_history: bool = False) -> dict:
        with self._lock:
            if job_id not in self._jobs:
                raise KeyError(f"Job '{job_id}' does not exist")
            out = copy.deepcopy(self._jobs[job_id])
            if embed_history:
                out["history"] = copy.deepcopy(self._history[job_id])
            return out

    def start_run(self, job_id: str) -> str:
        job = self.job(job_id)
        run_id = time.strftime("%Y%m%d%H%M%S") + uuid.uuid4().hex[:5]
        run = job.get("run", {})
        sandbox = tempfile.mkdtemp(prefix=f"job-{job_id}-", dir=os.path.join(self.cluster.work_dir))
        env = {k: os.environ[k] for k in ("PATH", "LANG", "TMPDIR") if k in os.environ}
        env.update({k: str(v) for k, v in (run.get("env") or {}).items() if not isinstance(v, dict)})
        env.update({"MESOS_SANDBOX": sandbox, "METRONOME_JOB_ID": job_id, "METRONOME_RUN_ID": run_id})
        proc = subprocess.Popen(["bash", "-c", run.get("cmd") or "true"], cwd=sandbox, env=env,
                                stdin=subprocess.DEVNULL, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                                start_new_session=True)
        with self._lock:
            self._active[f"{job_id}/{run_id}"] = proc
        started = time.time()

        def wait():
            out, _ = proc.communicate()
            rec = {"id": run_id, "createdAt": started, "finishedAt": time.time(),
                   "output": out.decode("utf-8", "replace")[-4096:]}
            with self._lock:
                self._active.pop(f"{job_id}/{run_id}", None)
                hist = self._history.get(job_id)
                if hist is not None:
                    hist["successfulFinishedRuns" if proc.returncode == 0 else "failedFinishedRuns"].append(rec)
        threading.Thread(target=wait, name=f"job-{job_id}-{run_id}", daemon=True).start()
        return run_id

    def shutdown(self) -> None:
        with self._lock:
            procs = list(self._active.values())
        for p in procs:
            try:
                p.kill()
            except OSError:
                pass
