"""argparse validators and task-splitting flags (reference ``shared_utils/util.py:371-506``)."""
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


def get_slurm_job_array_ids(parse_total_tasks_by_max_variable: bool = True, log_ids: bool = True,
                            verbose: bool = True,
                            task_index_remapping_json_file_path: Optional[str] = None) -> Tuple[int, int, int]:
    """``(job_id, total_tasks, task_index)`` of a SLURM job-array task (reference
    ``shared_utils/util.py:1120-1158``, U4): ``SLURM_ARRAY_TASK_ID`` + optional ``TASK_ID_OFFSET``,
    optionally remapped through a JSON list; total from ``TOTAL_TASKS``, else
    ``SLURM_ARRAY_TASK_MAX + 1`` (or ``SLURM_ARRAY_TASK_COUNT``)."""
    import json
    from .log import log
    job_id = int(os.environ["SLURM_ARRAY_JOB_ID"])
    task_index = int(os.environ["SLURM_ARRAY_TASK_ID"])
    if "TASK_ID_OFFSET" in os.environ:
        offset = int(os.environ["TASK_ID_OFFSET"])
        if verbose:
            log("Raw task index %d with offset %d." % (task_index, offset))
        task_index += offset
    if task_index_remapping_json_file_path is not None:
        with open(task_index_remapping_json_file_path) as f:
            remapped = int(json.load(f)[task_index])
        if verbose:
            log("Remapped task index %d into %d." % (task_index, remapped))
        task_index = remapped
    if "TOTAL_TASKS" in os.environ:
        total_tasks = int(os.environ["TOTAL_TASKS"])
    elif parse_total_tasks_by_max_variable:
        total_tasks = int(os.environ["SLURM_ARRAY_TASK_MAX"]) + 1
    else:
        total_tasks = int(os.environ["SLURM_ARRAY_TASK_COUNT"])
    if log_ids:
        log("Running job %s, task %d of %d." % (job_id, task_index, total_tasks))
    return job_id, total_tasks, task_index
