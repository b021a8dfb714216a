"""Timestamped, rank-aware logging helpers (reference ``shared_utils/util.py:24-79``: ``log``,
``start_log``, ``close_log``, ``restart_log`` (broken in the reference: it calls ``start_log()``
without arguments), ``log_file_open``, ``create_time_measure_if_verbose``)."""
from __future__ import annotations

import datetime
import os
import sys
from contextlib import contextmanager
from typing import Optional, TextIO

_LOG_FILE: Optional[TextIO] = None
_LOG_ARGS = None


def _rank() -> int:
    return int(os.environ.get("RANK", "0"))


def log(*message, end: str = "\n", all_ranks: bool = False) -> None:
    """Print a timestamped line (rank 0 only unless ``all_ranks``), tee'd to the open log file."""
    if not all_ranks and _rank() != 0:
        return
    text = "[%s] %s" % (datetime.datetime.now().strftime("%Y_%m_%d-%H:%M:%S"), " ".join(map(str, message)))
    print(text, end=end, flush=True)
    if _LOG_FILE is not None:
        _LOG_FILE.write(text + ("\n" if end == "\r" else end))
        _LOG_FILE.flush()


def start_log(log_dir: str, log_file_base_name: str) -> str:
    """Open ``<log_dir>/<base>__<pid>.txt`` (one file per process, as the reference)."""
    global _LOG_FILE, _LOG_ARGS
    os.makedirs(log_dir, exist_ok=True)
    path = os.path.join(log_dir, "%s__%d.txt" % (log_file_base_name, os.getpid()))
    _LOG_FILE = open(path, "w")
    _LOG_ARGS = (log_dir, log_file_base_name)
    log("Started log file %s" % path)
    return path


def close_log() -> None:
    global _LOG_FILE
    if _LOG_FILE is not None:
        _LOG_FILE.close()
        _LOG_FILE = None


def restart_log() -> Optional[str]:
    """Close and reopen the log with the arguments of the last :func:`start_log`."""
    close_log()
    if _LOG_ARGS is None:
        return None
    return start_log(*_LOG_ARGS)


def log_file_open() -> bool:
    return _LOG_FILE is not None


@contextmanager
def create_time_measure_if_verbose(opening_statement: str, verbose: bool):
    from .timing import TimeMeasure
    if verbose:
        with TimeMeasure(opening_statement):
            yield
    else:
        yield


def _stderr(*message) -> None:
    print(*message, file=sys.stderr, flush=True)
