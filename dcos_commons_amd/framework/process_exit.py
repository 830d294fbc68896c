"""Process exit codes (reference sdk/.../framework/ProcessExit.java:11-67).

Any unrecoverable scheduler error exits the process (no zombie state); the supervisor restarts it
and the scheduler resumes from the persisted state. Thread stacks are dumped before exiting.
"""
from __future__ import annotations

import faulthandler
import logging
import os
import signal
import sys
import threading

LOGGER = logging.getLogger(__name__)


class ProcessExitError(SystemExit):
    """Raised instead of exiting when ``ProcessExit.set_test_mode(True)``."""

    def __init__(self, code: int, cause=None):
        super().__init__(code)
        self.code = code
        self.cause = cause


class ProcessExit:
    SUCCESS = 0
    INITIALIZATION_FAILURE = 1
    REGISTRATION_FAILURE = 2
    DISCONNECTED = 5
    ERROR = 6
    DEADLOCK_ENCOUNTERED = 7
    LOCK_UNAVAILABLE = 8
    API_SERVER_ERROR = 9
    SCHEDULER_ALREADY_UNINSTALLING = 11
    DRIVER_EXITED = 13

    _test_mode = False

    @classmethod
    def set_test_mode(cls, enabled: bool) -> None:
        cls._test_mode = enabled

    @classmethod
    def exit(cls, code: int, cause: BaseException = None) -> None:
        if cause is not None:
            LOGGER.error("Process exiting with code %d: %s", code, cause)
        else:
            LOGGER.error("Process exiting with code %d", code)
        if cls._test_mode or os.environ.get("SDK_PROCESS_EXIT_RAISES"):
            raise ProcessExitError(code, cause)
        try:
            faulthandler.dump_traceback(file=sys.stderr, all_threads=True)
        except Exception:  # noqa: BLE001
            pass
        run_shutdown_hooks()
        logging.shutdown()
        os._exit(code)


# -- shutdown hooks (the JVM's Runtime.addShutdownHook: e.g. CuratorLocker releases the service lock
#    so the next scheduler does not wait for the ZooKeeper session to expire) ---------------------
_hooks = []
# re-entrant: the SIGTERM handler runs on the main thread, possibly while that same thread is inside
# add_shutdown_hook/run_shutdown_hooks; a plain Lock would deadlock the process there
_hooks_lock = threading.RLock()
_hooks_ran = False


def add_shutdown_hook(fn) -> None:
    """Registers ``fn`` once (a hook added again is not run twice)."""
    with _hooks_lock:
        if fn not in _hooks:
            _hooks.append(fn)


def run_shutdown_hooks() -> None:
    global _hooks_ran
    with _hooks_lock:
        if _hooks_ran:
            return
        _hooks_ran = True
        hooks = list(reversed(_hooks))
    for fn in hooks:
        try:
            fn()
        except Exception:  # noqa: BLE001
            LOGGER.exception("shutdown hook failed")


def install_signal_handlers() -> bool:
    """SIGTERM (what Marathon sends to roll or stop a scheduler) runs the shutdown hooks and exits
    with 143, as the JVM does. Only possible from the main thread; returns whether installed."""
    if threading.current_thread() is not threading.main_thread():
        return False

    def on_term(signum, frame):
        LOGGER.info("Received signal %d: running shutdown hooks and exiting", signum)
        run_shutdown_hooks()
        logging.shutdown()
        os._exit(128 + signum)
    signal.signal(signal.SIGTERM, on_term)
    return True
