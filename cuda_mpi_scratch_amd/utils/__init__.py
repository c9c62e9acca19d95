"""Utilities: launcher environment, timers, per-rank logging, JSON metrics."""
from .env import local_rank, local_size, select_device, world_rank, world_size  # noqa: F401
from .log import hostname, is_quiet, rank_print, set_quiet  # noqa: F401
from .metrics import append_json, device_info, git_sha, record  # noqa: F401
from .timer import DeviceTimer, Summary, WallTimer, summarize  # noqa: F401
