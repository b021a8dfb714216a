"""argparse validators and task-splitting flags (reference ``shared_utils/util.py:371-506``).

The reference's SLURM job-array helper (``shared_utils/util.py:1120-1158``) is not provided: SURVEY
marks it "not needed" -- ranks come from the ``torchrun`` environment, and task splitting from
``--task-index`` / ``--total-tasks`` or ``SLURM_ARRAY_TASK_ID`` (:func:`determine_parser_task_details`)."""
from __future__ import annotations

import argparse
import os
from typing import Optional, Tuple


def get_parser_bool_type(parser: argparse.ArgumentParser):
    def _bool(value: str) -> bool:
        v = value.lower()
        if v in ("yes", "true", "t", "y", "1"):
            return True
        if v in ("no", "false", "f", "n", "0"):
            return False
        parser.error("%r is not a boolean" % value)
    return _bool


def get_parser_file_type(parser: argparse.ArgumentParser, must_exist: bool = False):
    def _file(path: str) -> str:
        if must_exist and not os.path.isfile(path):
            parser.error("file %s does not exist" % path)
        parent = os.path.dirname(os.path.abspath(path))
        if not os.path.isdir(parent):
            parser.error("directory %s does not exist" % parent)
        return path
    return _file


def get_parser_directory_type(parser: argparse.ArgumentParser, create_if_not_exists: bool = False):
    def _dir(path: str) -> str:
        if not os.path.isdir(path):
            if create_if_not_exists:
                os.makedirs(path, exist_ok=True)
            else:
                parser.error("directory %s does not exist" % path)
        return path
    return _dir


def add_parser_task_arguments(parser: argparse.ArgumentParser) -> None:
    """``--task-index``/``--total-tasks`` split a job into independent tasks (e.g. SLURM arrays);
    defaults come from ``SLURM_ARRAY_TASK_ID``/``TASK_ID_OFFSET``/``TOTAL_TASKS`` when set."""
    parser.add_argument("--task-index", type=int, default=None)
    parser.add_argument("--total-tasks", type=int, default=None)


def determine_parser_task_details(args) -> Tuple[int, int]:
    task_index: Optional[int] = getattr(args, "task_index", None)
    total_tasks: Optional[int] = getattr(args, "total_tasks", None)
    if task_index is None and "SLURM_ARRAY_TASK_ID" in os.environ:
        task_index = int(os.environ["SLURM_ARRAY_TASK_ID"]) + int(os.environ.get("TASK_ID_OFFSET", "0"))
    if total_tasks is None and "TOTAL_TASKS" in os.environ:
        total_tasks = int(os.environ["TOTAL_TASKS"])
    task_index = 0 if task_index is None else task_index
    total_tasks = 1 if total_tasks is None else total_tasks
    if not 0 <= task_index < total_tasks:
        raise ValueError("task index %d out of range for %d tasks" % (task_index, total_tasks))
    return task_index, total_tasks

