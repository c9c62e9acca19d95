"""Workloads ("model families") of the suite: 2D stencil, ping-pong, dot product."""
from .dot import DotProduct  # noqa: F401
from .pingpong import PingPong, parse_sweep, reference_report  # noqa: F401
from .stencil2d import Stencil2D, StencilConfig, format_tile  # noqa: F401
