"""Metronome jobs (reference: testing/sdk_jobs.py) on the local cluster's Metronome stand-in."""
from __future__ import annotations

import json
import logging
import time
from typing import Any, Dict, List

LOG = logging.getLogger(__name__)


def _metronome():
    from dcos_commons_amd.testing.cluster import current

    return current().metronome


def install_job(job_dict: Dict[str, Any]) -> None:
    _remove_job_by_name(job_dict["id"])   # replace any job of that name
    LOG.info("Adding job %s:\n%s", job_dict["id"], json.dumps(job_dict))
    _metronome().add_job(job_dict)


def remove_job(job_dict: Dict[str, Any]) -> None:
    _remove_job_by_name(job_dict["id"])


def _remove_job_by_name(job_name: str) -> None:
    try:
        _metronome().remove_job(job_name, stop_current_runs=True)
    except KeyError:
        pass


class InstallJobContext:
    """Installs the jobs for the duration of a ``with`` block."""

    def __init__(self, jobs: List[Dict[str, Any]]) -> None:
        self.job_dicts = jobs

    def __enter__(self) -> None:
        for j in self.job_dicts:
            install_job(j)

    def __exit__(self, *args: Any) -> None:
        for j in self.job_dicts:
            remove_job(j)


def run_job(job_dict: Dict[str, Any], timeout_seconds: int = 600, raise_on_failure: bool = True) -> str:
    """Starts a run and waits for it to show up among the job's successful runs."""
    job_name = job_dict["id"]
    run_id = _metronome().start_run(job_name)
    LOG.info("Started job %s: run id %s", job_name, run_id)
    deadline = time.time() + timeout_seconds
    while True:
        history = _metronome().job(job_name, embed_history=True)["history"]
        if raise_on_failure and run_id in [r["id"] for r in history["failedFinishedRuns"]]:
            out = next(r["output"] for r in history["failedFinishedRuns"] if r["id"] == run_id)
            raise Exception(f"Job {job_name} with id {run_id} has failed, exiting early:\n{out}")
        if run_id in [r["id"] for r in history["successfulFinishedRuns"]] + \
                ([] if raise_on_failure else [r["id"] for r in history["failedFinishedRuns"]]):
            return run_id
        if time.time() >= deadline:
            raise TimeoutError(f"Job {job_name} run {run_id} did not finish within {timeout_seconds}s")
        time.sleep(0.1)


class RunJobContext:
    """Runs ``before_jobs`` on entry and ``after_jobs`` on exit (each installed for the run)."""

    def __init__(self, before_jobs: List[Dict[str, Any]] = (), after_jobs: List[Dict[str, Any]] = (),
                 timeout_seconds: int = 600) -> None:
        self.before_jobs, self.after_jobs, self.timeout_seconds = list(before_jobs), list(after_jobs), timeout_seconds

    def __enter__(self) -> None:
        for j in self.before_jobs:
            with InstallJobContext([j]):
                run_job(j, timeout_seconds=self.timeout_seconds)

    def __exit__(self, *args: Any) -> None:
        for j in self.after_jobs:
            with InstallJobContext([j]):
                run_job(j, timeout_seconds=self.timeout_seconds)
