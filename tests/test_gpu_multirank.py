"""The native multi-rank solver on ONE GPU: N processes share the device and
exchange halos through the IPC backend (HIP IPC mappings + device-side ready /
free counters), so the whole multi-rank schedule — per-peer plan, pack, put,
wait, unpack, overlap with the interior, hipGraph replay, time blocking — runs
on real hardware, checked against the whole-grid reference."""
import pytest
import torch

from cuda_mpi_scratch_amd.ops import jacobi_reference_global, random_values
from tests.mp_util import run_ranks, run_ranks_raw

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,dims,time_block,overlap,graph", [
    (2, "1x2", 12, True, True),
    (2, "2x1", 4, False, False),
    (4, "2x2", 12, True, True),
    (4, "2x2", 1, True, False),
    (6, "2x3", 5, True, True),
    (8, "4x2", 20, False, True),  # the 8-GPU grid at the production depth: 8 ranks' agreements
])
def test_ipc_solver_matches_global_reference(gpu, n, dims, time_block, overlap, graph):
    w, h, iters, seed = 264, 200, 29, 7
    res = run_ranks("gpu_solver", n, {"w": w, "h": h, "dims": dims, "iters": iters, "seed": seed,
                                      "time_block": time_block, "overlap": overlap, "graph": graph}, gpu=True)
    assert all(r["native"] and r["backend"] == "ipc" for r in res), res
    if graph:
        assert all(r["graph"] == "captured" for r in res)
    got = torch.tensor(res[0]["grid"], dtype=torch.float64)
    ref = jacobi_reference_global(random_values(0, 0, w, h, w, seed), iters).double()
    assert (got - ref).abs().max().item() < 1e-5


def test_ipc_solver_f64_bitwise_vs_single_rank(gpu):
    """Decomposition invariance on the GPU: 4 IPC ranks == 1 rank, bitwise (f64)."""
    args = {"w": 200, "h": 136, "iters": 25, "seed": 3, "dtype": "f64", "time_block": 12}
    one = run_ranks("gpu_solver", 1, dict(args, dims="1x1"), gpu=True)
    four = run_ranks("gpu_solver", 4, dict(args, dims="2x2"), gpu=True)
    assert torch.equal(torch.tensor(one[0]["grid"]), torch.tensor(four[0]["grid"]))


@pytest.mark.parametrize("n,dims,dtype,time_block,runs", [
    (2, "1x2", "f32", 20, [20, 20]),      # fp32 default S: two-stage pipeline, left/right pushes
    (2, "2x1", "f32", 20, [7, 33]),       # up/down pushes, left/right self copies; odd splits
    (4, "2x2", "f32", 12, [29]),          # corners through the diagonal neighbour
    (6, "2x3", "f64", 16, [16, 16]),      # fp64 wide-lane pipeline
    (4, "2x2", "f32", 5, [11]),           # bands of 5 columns: 4-byte push path
    (2, "1x2", "f32", 1, [6]),            # one push per iteration
])
def test_ipc_direct_halo_matches_global_reference(gpu, n, dims, dtype, time_block, runs):
    """Device-initiated halo (IPC backend, direct mode): each pass pushes its
    edge bands into the neighbours' ghost rings; several run() calls re-prime."""
    w, h, seed = 272, 216, 13
    iters = sum(runs)
    res = run_ranks("gpu_solver", n, {"w": w, "h": h, "dims": dims, "iters": iters, "runs": runs, "seed": seed,
                                      "dtype": dtype, "time_block": time_block, "direct": True}, gpu=True)
    assert all(r["backend"] == "ipc" and "IPC direct push" in r["halo"] for r in res), res
    got = torch.tensor(res[0]["grid"], dtype=torch.float64)
    ref = jacobi_reference_global(random_values(0, 0, w, h, w, seed, dtype=torch.float64), iters)
    assert (got - ref).abs().max().item() < (1e-5 if dtype == "f32" else 1e-12)


@pytest.mark.parametrize("dtype,time_block", [("f32", 20), ("f64", 16)])
def test_ipc_ranks_unequal_coefficients_scaled_form(gpu, dtype, time_block):
    """Unequal coefficients across ranks (IPC, 2 x 2, direct halo): every rank
    runs the scaled form and the field stays within rounding of the fp64
    reference of the same weights."""
    w, h, seed, runs = 272, 216, 17, [time_block, 2 * time_block]
    res = run_ranks("gpu_solver", 4, {"w": w, "h": h, "dims": "2x2", "iters": sum(runs), "runs": runs, "seed": seed,
                                      "dtype": dtype, "time_block": time_block, "direct": True,
                                      "c_center": 0.5, "c_neighbor": 0.125}, gpu=True)
    assert all(r["fast_form"] and r["scaled_form"] for r in res), res
    got = torch.tensor(res[0]["grid"], dtype=torch.float64)
    ref = jacobi_reference_global(random_values(0, 0, w, h, w, seed, dtype=torch.float64), sum(runs), 0.5, 0.125)
    assert (got - ref).abs().max().item() < (2e-6 if dtype == "f32" else 1e-13)


@pytest.mark.parametrize("engine", ["kernel", "copy-engine"])
def test_ipc_direct_halo_bitwise_vs_classic_exchange(gpu, engine):
    """The push (by a CU kernel, or by the SDMA copy engines: one
    hipMemcpy2DAsync per band) and the pack -> put -> unpack exchange deliver
    the same ghost cells: identical results, bit for bit (4 ranks, 2 x 2)."""
    args = {"w": 264, "h": 200, "dims": "2x2", "iters": 40, "seed": 4, "time_block": 20, "overlap": False}
    direct = run_ranks("gpu_solver", 4, dict(args, direct=True, direct_engine=engine), gpu=True)
    classic = run_ranks("gpu_solver", 4, dict(args, direct=False), gpu=True)
    assert "IPC direct push" in direct[0]["halo"] and "IPC direct push" not in classic[0]["halo"]
    assert ("SDMA copy engines" in direct[0]["halo"]) == (engine == "copy-engine")
    assert torch.equal(torch.tensor(direct[0]["grid"]), torch.tensor(classic[0]["grid"]))


def test_copy_engine_direct_halo_validated(gpu):
    """The copy-engine push behind the validation gate (three super-steps from
    a poisoned ring, bitwise against the IPC exchange, then timed): bitwise
    equal on every rank, whatever the timing decides; the field stays exact."""
    w, h, seed, runs = 272, 216, 29, [20, 20]
    res = run_ranks("gpu_solver", 2, {"w": w, "h": h, "dims": "1x2", "iters": sum(runs), "runs": runs, "seed": seed,
                                      "time_block": 20, "overlap": False, "direct": "validate",
                                      "direct_engine": "copy-engine", "prepare": 20, "comm_timeout": 60}, gpu=True)
    states = [r["direct_state"] for r in res]
    assert states[0].startswith(("validated: bitwise equal", "rejected (slower): bitwise equal")), states
    got = torch.tensor(res[0]["grid"], dtype=torch.float64)
    ref = jacobi_reference_global(random_values(0, 0, w, h, w, seed), sum(runs)).double()
    assert (got - ref).abs().max().item() < 1e-5


def test_one_rank_reading_its_field_keeps_ranks_in_step(gpu):
    """Reading a field marks it changed on that rank only; the priming exchange
    of the next run must still be issued by every rank (it is collective), so
    ranks whose callers differ stay matched (post-exchange schedule, 3 runs)."""
    w, h, seed, runs = 264, 200, 9, [20, 20, 13]
    res = run_ranks("gpu_solver", 2, {"w": w, "h": h, "dims": "1x2", "iters": sum(runs), "runs": runs, "seed": seed,
                                      "time_block": 20, "overlap": False, "direct": False, "rank0_reads": True},
                    gpu=True)
    assert all(r["native"] and r["backend"] == "ipc" for r in res), res
    got = torch.tensor(res[0]["grid"], dtype=torch.float64)
    ref = jacobi_reference_global(random_values(0, 0, w, h, w, seed), sum(runs)).double()
    assert (got - ref).abs().max().item() < 1e-5


@pytest.mark.parametrize("time_block", [20, 1])
def test_peers_exchange_once_per_super_step(gpu, time_block):
    """With peers a run of n super-steps issues exactly n exchanges: the priming
    one, then one after every pass but the last (the next run primes anyway).
    The 20-step window bench.py times at N = 8 is one exchange + one pass."""
    w, h, seed = 264, 200, 13
    runs = [45, 20, 7] if time_block > 1 else [3, 1, 2]
    res = run_ranks("gpu_solver", 2, {"w": w, "h": h, "dims": "1x2", "iters": sum(runs), "runs": runs, "seed": seed,
                                      "time_block": time_block, "overlap": False, "direct": False}, gpu=True)
    for r in res:
        assert r["native"] and r["backend"] == "ipc", r
        assert all(ex == steps for ex, steps in r["exchanges"]), r["exchanges"]
    assert [s for _, s in res[0]["exchanges"]] == [-(-n // time_block) for n in runs]
    got = torch.tensor(res[0]["grid"], dtype=torch.float64)
    ref = jacobi_reference_global(random_values(0, 0, w, h, w, seed), sum(runs)).double()
    assert (got - ref).abs().max().item() < 1e-5


@pytest.mark.parametrize("n,dims,w,h,steady", [(2, "1x2", 8192, 1024, "serial"),
                                               (2, "2x1", 4096, 2048, "interior-first"),
                                               (4, "2x2", 8192, 2048, "interior-first"),
                                               (4, "2x2", 8192, 2048, "auto")])
def test_ipc_interior_first_bitwise_vs_serial(gpu, n, dims, w, h, steady):
    """The interior-first schedule on the IPC exchange (ranks sharing one GPU;
    4096 x 1024 tiles, so the chunk-list form exists): the inner chunks run on
    the side stream while pack, put, wait and unpack run on main, then the
    ghost-ring chunks. Only the order of the work changes, so the global field
    is bitwise the serial schedule's (compared by digest); with steady =
    interior-first every super-step of a call runs that way; steady = auto
    (prepare() of a 3-super-step window) runs the steady decision over the
    ranks, which all adopt the same schedule."""
    runs = [20, 60, 13]
    args = {"w": w, "h": h, "dims": dims, "iters": sum(runs), "runs": runs, "seed": 31, "time_block": 20,
            "overlap": False, "direct": False, "digest": True}
    extra = {"prepare": 60, "comm_timeout": 120} if steady == "auto" else {}
    first = run_ranks("gpu_solver", n, dict(args, opening="interior-first", steady=steady, **extra), gpu=True)
    serial = run_ranks("gpu_solver", n, dict(args, opening="serial", steady="serial"), gpu=True)
    chosen = {r["choice"]["steady"] for r in first}
    assert len(chosen) == 1, chosen
    took = chosen.pop()
    assert took == steady or (steady == "auto" and took in ("serial", "interior-first")), took
    for r in first:
        assert r["backend"] == "ipc" and r["halo_last"], (r["halo_modes"], r["choice"]["opening"])
        assert r["choice"]["opening"] == "interior-first", r["choice"]
        if steady == "auto":
            assert f"over {n} rank(s)" in r["choice"]["steady_reason"], r["choice"]["steady_reason"]
        assert all(ex == steps for ex, steps in r["exchanges"]), r["exchanges"]  # one exchange per super-step
        assert "interior-first" in r["halo_modes"][1], r["halo_modes"]
        assert ("every super-step interior-first" in r["halo_modes"][1]) == (took == "interior-first")
    assert all(not r["halo_last"] for r in serial)
    assert first[0]["digest"] == serial[0]["digest"]
    assert 0.0 < first[0]["absmax"] <= 1.0  # a bounded operator on a field in [0, 1)


@pytest.mark.parametrize("n,dims,w,h", [(4, "2x2", 8192, 2048), (8, "4x2", 8192, 4096)])
def test_ipc_ranks_agree_on_measured_schedules(gpu, n, dims, w, h):
    """opening = auto, steady = auto with 4 or 8 ranks (4096 x 1024 tiles; 4 x 2
    is the 8-GPU grid) on the IPC exchange: prepare() runs the multi-rank
    decisions the 8-GPU bench runs (per-round maxima over ranks through the
    host allgather, the same samples on every rank), every rank adopts the same
    opening and steady schedule, and the field is bitwise the serial schedule's
    whatever they chose."""
    runs = [40, 20]
    args = {"w": w, "h": h, "dims": dims, "iters": sum(runs), "runs": runs, "seed": 37, "time_block": 20,
            "overlap": False, "direct": False, "digest": True, "comm_timeout": 120}
    res = run_ranks("gpu_solver", n, dict(args, prepare=40), gpu=True)
    serial = run_ranks("gpu_solver", n, dict(args, opening="serial", steady="serial"), gpu=True)
    choices = [(r["choice"]["opening"], r["choice"]["steady"]) for r in res]
    assert len(set(choices)) == 1, choices
    opening, steady = choices[0]
    assert opening in ("serial", "interior-first") and steady in ("serial", "interior-first"), choices
    for r in res:
        assert "host allgather" in r["agreement"], r["agreement"]
        assert f"{n} rank" in r["choice"]["reason"] or r["choice"]["reason"].startswith("no rank"), r["choice"]["reason"]
        if opening == "interior-first":
            assert f"over {n} rank(s)" in r["choice"]["steady_reason"], r["choice"]
        assert all(ex == steps for ex, steps in r["exchanges"]), r["exchanges"]
    assert res[0]["digest"] == serial[0]["digest"]
    print(f"{n} ranks chose opening {opening}, steady {steady}: {res[0]['choice']['reason']}")


@pytest.mark.parametrize("fail_rank", [None, 2])
def test_device_barrier_falls_back_to_the_host_allgather(gpu, fail_rank):
    """The device barrier in front of every timed decision sample (VERDICT r05
    item 5). Four IPC ranks sharing the GPU, each given a one-rank RCCL
    loopback communicator for the barrier only (RCCL refuses two ranks of one
    communicator on one GPU). The first barrier probes RCCL on every rank and
    the ranks agree through the host allgather: all good -> "rccl all-reduce"
    everywhere; one rank's barrier failing (fault injection) -> every rank
    takes the host allgather, prepare() completes, the decisions still agree,
    and the field is bitwise the serial schedule's."""
    runs = [20]
    args = {"w": 8192, "h": 2048, "dims": "2x2", "iters": sum(runs), "runs": runs, "seed": 41, "time_block": 20,
            "overlap": False, "direct": False, "digest": True, "comm_timeout": 60}
    res = run_ranks("gpu_solver", 4, dict(args, prepare=20, barrier_loopback=True, barrier_fail_rank=fail_rank),
                    gpu=True)
    paths = [r["barrier_path"] for r in res]
    if fail_rank is None:
        assert paths == ["rccl all-reduce"] * 4, paths
    else:
        assert all(p.startswith("host allgather (fallback: the RCCL barrier failed on") for p in paths), paths
        assert "injected RCCL barrier failure" in paths[fail_rank], paths
        assert all("another rank" in p for i, p in enumerate(paths) if i != fail_rank), paths
    assert len({r["choice"]["opening"] for r in res}) == 1, [r["choice"] for r in res]
    assert all(r["choice"]["opening"] in ("serial", "interior-first") for r in res)
    serial = run_ranks("gpu_solver", 4, dict(args, opening="serial", steady="serial"), gpu=True)
    assert res[0]["digest"] == serial[0]["digest"]


@pytest.mark.parametrize("direct", [True, False])
def test_ipc_warm_and_prepare_leave_the_state_alone(gpu, direct):
    """bench.py's prepare() + warm() on the IPC paths (device-initiated pushes and
    the classic pack -> put -> unpack) launch real passes and exchanges but must
    not advance the field: the result equals the plain run's reference."""
    w, h, seed, runs = 272, 216, 19, [20, 20]
    res = run_ranks("gpu_solver", 2, {"w": w, "h": h, "dims": "1x2", "iters": sum(runs), "runs": runs, "seed": seed,
                                      "time_block": 20, "overlap": False, "direct": direct, "prepare": 20, "warm": 20},
                    gpu=True)
    assert all(r["backend"] == "ipc" and ("IPC direct push" in r["halo"]) == direct for r in res), res
    got = torch.tensor(res[0]["grid"], dtype=torch.float64)
    ref = jacobi_reference_global(random_values(0, 0, w, h, w, seed), sum(runs)).double()
    assert (got - ref).abs().max().item() < 1e-5


@pytest.mark.parametrize("direct", [True, False])
def test_rank_stalled_in_prepare_fails_the_job_within_the_watchdog(gpu, direct):
    """Fault injection: rank 1 stalls 40 s on entering prepare()
    (after a first run, as bench.py's warm-up leaves it). Rank 0's waits with
    collectives in flight are under the watchdog (5 s): it must fail well
    before the stalled rank wakes, naming the phase, instead of hanging."""
    args = {"w": 264, "h": 200, "dims": "1x2", "iters": 20, "seed": 5, "time_block": 20, "overlap": False,
            "direct": direct, "warmup_first": 20, "prepare": 20, "comm_timeout": 5,
            "stall": {"rank": 1, "phase": "prepare", "seconds": 40}}
    res = run_ranks_raw("gpu_solver", 2, args, timeout=200, gpu=True)
    r0 = res[0]
    assert r0["rc"] != 0, r0["stdout"][-2000:]
    assert "prepare" in r0["stderr"] and "timed out" in r0["stderr"], r0["stderr"][-3000:]
    assert r0["seconds"] < 40, r0["seconds"]  # failed on its own, not when the peer woke
    assert "[fault-inject] stalling" in res[1]["stderr"]


@pytest.mark.parametrize("fault", [None, "mismatch", "skip_wait"])
def test_direct_halo_validation_and_fallback(gpu, fault):
    """DirectHalo validate (the mode that lets the device-initiated push run
    between GPUs): prepare() runs three super-steps through the backend (here
    the IPC transport: ranks share the GPU) and three through the direct push
    from a sentinel-filled ring, compares the whole tiles bitwise on every rank
    and times both. Equal everywhere: validated (used if faster) or rejected as
    slower, on every rank alike. One rank's corrupted cell, or one rank's
    skipped wait for its neighbours' pushes (the visibility race the check
    guards; fault injection): every rank rejects it and keeps the backend. The
    field is exact either way, and the agreements went through the host
    allgather."""
    w, h, seed, runs = 272, 216, 23, [20, 20, 7]
    res = run_ranks("gpu_solver", 2, {"w": w, "h": h, "dims": "1x2", "iters": sum(runs), "runs": runs, "seed": seed,
                                      "time_block": 20, "overlap": False, "direct": "validate", "prepare": 20,
                                      "mismatch_rank": 1 if fault == "mismatch" else None,
                                      "skip_wait_rank": 0 if fault == "skip_wait" else None,
                                      "comm_timeout": 60}, gpu=True)
    states = [r["direct_state"] for r in res]
    assert len({s.split(":")[0] for s in states}) == 1, states  # one collective decision
    assert all(r["agreement"] == "host allgather" for r in res)
    if fault:
        assert states[0].startswith("rejected: the direct push differs"), states
        assert not any(r["direct"] for r in res)
    else:
        assert states[0].startswith(("validated: bitwise equal", "rejected (slower): bitwise equal")), states
        assert all(r["direct"] == states[0].startswith("validated") for r in res)
        if res[0]["direct"]:
            assert "IPC direct push" in res[0]["halo"]
            # A one-super-step call with the direct halo: the priming push, then a bare pass.
            assert all(r["exchanges"][0] == [1, 1] for r in res), res[0]["exchanges"]
    got = torch.tensor(res[0]["grid"], dtype=torch.float64)
    ref = jacobi_reference_global(random_values(0, 0, w, h, w, seed), sum(runs)).double()
    assert (got - ref).abs().max().item() < 1e-5


def test_bench_isolated_ipc_pingpong_two_ranks(gpu):
    """bench.py's N >= 2 IPC ping-pong runs in two child processes with their own
    rendezvous (here both on this GPU): rank 0's record gets the latency, the
    bandwidths and the verification, the ranks' own processes never touch it."""
    res = run_ranks("ipc_pingpong_isolated", 2, {"max_bytes": 1 << 20}, gpu=True, timeout=300)
    ex = res[0]["extras"]
    assert "pingpong_ipc_error" not in ex, ex
    assert ex["pingpong_ipc_device_8B_latency_us"] > 0 and ex["pingpong_ipc_device_1MiB_gbps"] > 0
    assert ex["pingpong_ipc_verified"] is True and "isolated" in ex["pingpong_ipc"]
    # The copy-engine transport, in the same isolation: latency, rates, both
    # directions and the overlap speedup of its largest message.
    assert "pingpong_peer_copy_error" not in ex, ex
    assert ex["pingpong_peer_copy_async_8B_latency_us"] > 0 and ex["pingpong_peer_copy_async_1MiB_gbps"] > 0
    assert ex["pingpong_peer_copy_bidir_1MiB_both_directions_gbps"] > 0
    assert ex["pingpong_peer_copy_verified"] is True
    assert res[1]["extras"] == {}


@pytest.mark.parametrize("mode", ["blocking", "async", "bidir", "overlap"])
def test_peer_copy_pingpong_two_processes(gpu, mode):
    """The copy-engine transport between two processes (here sharing the GPU):
    SDMA copies into the peer's IPC-mapped mailbox, flags published by one-lane
    kernels. Every size echoes bitwise (bidirectional: each side received the
    other's payload); the overlap mode reports all three timings, and the copy
    engine hides the transfer behind the ALU-bound kernel at least as well as
    running them one after the other."""
    sizes = [8, 4096, 1 << 20, 16 << 20]
    res = run_ranks("pingpong", 2, {"transport": "peer-copy", "sizes": sizes, "mode": mode}, gpu=True, timeout=300)
    for r in res:
        recs = r["records"]
        assert [x["bytes"] for x in recs] == sizes
        assert all(x["passed"] for x in recs), recs
    r0 = res[0]["records"]
    assert all(x["rtt_us"] > 0 and x["gbps"] > 0 for x in r0), r0
    if mode == "overlap":
        big = r0[-1]
        assert big["comm_alone_us"] > 0 and big["compute_alone_us"] > 0 and big["overlapped_us"] > 0
        assert big["overlapped_us"] < 1.05 * (big["comm_alone_us"] + big["compute_alone_us"]), big
