"""Process exit codes (reference sdk/.../framework/ProcessExit.java:11-67).

Any unrecoverable scheduler error exits the process (no zombie state); the supervisor restarts it
and the scheduler resumes from the persisted state. Thread stacks are dumped before exiting.
"""
from __future__ import annotations

import faulthandler
import logging
import os
import sys

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
        logging.shutdown()
        os._exit(code)
