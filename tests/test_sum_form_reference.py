"""The sum-form reference (the exact association of the GPU sum bodies) agrees
with the per-step Jacobi to rounding: few ulp over a pass, for fp32 and fp64."""
import pytest
import torch

from cuda_mpi_scratch_amd.ops import jacobi_reference_global, jacobi_sum_reference_global


@pytest.mark.parametrize("dtype,steps,tol", [(torch.float64, 16, 1e-14), (torch.float32, 20, 2e-6),
                                             (torch.float32, 32, 2e-6)])
def test_sum_form_reference_close_to_per_step(dtype, steps, tol):
    u = torch.rand(48, 72, generator=torch.Generator().manual_seed(steps), dtype=torch.float64).to(dtype)
    a = jacobi_sum_reference_global(u, steps)
    b = jacobi_reference_global(u, steps)
    assert (a.double() - b.double()).abs().max().item() <= tol


def test_sum_form_reference_is_one_scaled_pass():
    """S levels of plain sums then one multiply: with c = 1 it is the raw
    5-point sum recurrence (integers stay exact)."""
    u = torch.randint(0, 4, (8, 12), dtype=torch.int64).double()
    v = jacobi_sum_reference_global(u, 3, c=1.0)
    w = u.clone()
    for _ in range(3):
        w = w + torch.roll(w, 1, 0) + torch.roll(w, -1, 0) + torch.roll(w, 1, 1) + torch.roll(w, -1, 1)
    assert torch.equal(v, w)
