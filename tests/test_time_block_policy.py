"""The measured time-block policy (kernels::auto_time_block), host-side: the
values the tuner runs chose (docs/PERF.md, profiles/r02_sum), so a change to
the rule shows up as a test diff next to its measurements."""
import pytest


def _hip():
    try:
        from cuda_mpi_scratch_amd import hip

        return hip()
    except Exception as e:  # noqa: BLE001 - extension not built in this environment
        pytest.skip(f"HIP extension not importable: {e}")


@pytest.mark.parametrize(
    "w,h,dtype,sum_form,expected",
    [
        (32768, 32768, "f32", True, 24),   # >= 2^30 cells: S = 24 (37 joint groups) 11.1 vs 10.9 T at 20
        (32768, 32768, "f32", False, 20),  # per-step form
        (32768, 16384, "f32", True, 20),   # 2-GPU tile: 36 vs 37 joint groups
        (16384, 16384, "f32", True, 20),   # 4-GPU tile
        (16384, 8192, "f32", True, 20),    # 8-GPU tile: 18 joint groups at S = 20, 19 at 24
        (8192, 8192, "f32", True, 20),     # 9 joint groups at 20, 10 at 24 (8.6-8.9 vs 8.4 T)
        (4096, 2048, "f32", True, 24),     # 5 joint groups either way: the deeper block
        (8192, 8192, "f64", True, 16),     # wide-lane pipeline 8 + 8
        (8192, 8192, "f64", False, 12),    # per-step 6 + 6
        (512, 512, "f32", True, 12),       # small tiles: single-wave kernels
        (1 << 20, 1024, "f32", True, 24),  # 4 MiB rows: the pipelines walk shares in descriptor-sized pieces
        (9_000_000, 64, "f32", True, 16),  # rows beyond ~8.3 M fp32 columns: no 64-row piece fits the descriptor
    ],
)
def test_auto_time_block(w, h, dtype, sum_form, expected):
    assert _hip().auto_time_block(w, h, dtype, sum_form) == expected


def test_twenty_steps_at_block_24_run_as_one_pass():
    """run(K) splits K into ceil(K / S) near-equal super-steps: the driver's
    20-step window at S = 24 is one pass of 20 (mirrors StencilSolver::split)."""
    def split(iters, block):
        blocks = (iters + block - 1) // block
        base, extra = divmod(iters, blocks)
        return sorted([base + 1] * extra + [base] * (blocks - extra), reverse=True)

    assert split(20, 24) == [20]
    assert split(40, 24) == [20, 20]
    assert split(240, 24) == [24] * 10
    assert split(30, 20) == [15, 15]
