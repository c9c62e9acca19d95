"""Device ops: thin wrappers over the gfx950 HIP kernels (csrc/kernels), with
exact CPU reference implementations for CPU tensors."""
from .dot import DotWorkspace, dot  # noqa: F401
from .fill import fill, fill_random, fill_region, random_values  # noqa: F401
from .stencil import (box_reference, jacobi_reference_global, jacobi_sum_reference_global,  # noqa: F401
                      stencil5, stencil5_rect, stencil5_reference, stencil_box)
