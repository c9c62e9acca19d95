"""Distributed runtime: torch.distributed bootstrap, Cartesian decomposition,
halo-exchange backends (native RCCL / torch P2P / local)."""
from .cart import Decomposition, choose_dims, parse_dims  # noqa: F401
from .dist import DistContext, init, make_rccl_comm  # noqa: F401
from .watchdog import CommTimeout, CommWatchdog  # noqa: F401
from .halo import NativeHalo, TorchHalo, make_plan, region_view, tile_view  # noqa: F401
