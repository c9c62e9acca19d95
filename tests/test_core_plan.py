"""Host-side core (C++ via _mxs_core): regions, topology, halo-plan symmetry."""
import itertools
import os
import subprocess

import pytest

import cuda_mpi_scratch_amd as pkg

C = pkg.core()


def test_cpp_unit_tests(build_dir):
    exe = os.path.join(build_dir, "mxs_unit_tests")
    if not os.path.exists(exe):
        pytest.skip("C++ unit tests not built")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    assert "all passed" in r.stdout


def test_debug_bounds_accessor(build_dir):
    """-DMXS_DEBUG_BOUNDS build: in-window accesses pass, one past the core aborts loudly."""
    exe = os.path.join(build_dir, "mxs_bounds_test")
    if not os.path.exists(exe):
        pytest.skip("bounds test not built")
    ok = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert ok.returncode == 0 and "sum 276" in ok.stdout
    bad = subprocess.run([exe, "oob"], capture_output=True, text=True, timeout=60)
    assert bad.returncode != 0 and "(6, 0) outside the window" in bad.stderr


def test_region_text_format():
    g = C.Array2D(20, 20, 20)
    core = C.sub_array_region(g, 5, 5, C.RegionID.CENTER)
    assert str(core) == "width:  16, height: 16, x offset: 2, y offset: 2"
    assert str(C.sub_array_region(core, 5, 5, C.RegionID.TOP)) == "width:  16, height: 2, x offset: 2, y offset: 2"
    assert int(C.RegionID.BOTTOM_RIGHT) == 8 and int(C.RegionID.RIGHT) == 12


def test_dims_and_split():
    assert C.dims_create(8) == (4, 2)
    assert C.dims_create(9) == (3, 3)
    assert C.dims_create(12) == (4, 3)
    starts = [C.block_split(10, 3, i) for i in range(3)]
    assert starts == [(0, 4), (4, 3), (7, 3)]


def test_cart_grid_text_and_shift():
    t = C.CartTopology(3, 3)
    assert t.grid_text() == "0 1 2 \n3 4 5 \n6 7 8 \n"
    np_ = C.CartTopology(3, 3, False, False)
    assert np_.cart_shift(4, 0, 1) == (1, 7) and np_.cart_shift(4, 1, 1) == (3, 5)
    assert np_.cart_shift(0, 0, 1) == (C.PROC_NULL, 3)


GRIDS = [(1, 1), (1, 2), (2, 1), (2, 2), (2, 4), (4, 2), (3, 3), (1, 3), (3, 5)]


@pytest.mark.parametrize("rows,cols", GRIDS)
@pytest.mark.parametrize("periodic", [True, False])
@pytest.mark.parametrize("corners", [True, False])
def test_plan_symmetry(rows, cols, periodic, corners):
    """What rank r sends to p equals, segment by segment, what p expects from r."""
    topo = C.CartTopology(rows, cols, periodic, periodic)
    g = C.TileGeom.aligned(13, 7, 2, 2, 4)
    plans = [C.make_halo_plan(topo, r, g, corners, False) for r in range(rows * cols)]
    for r, p in enumerate(plans):
        assert sum(m.count for m in p.sends) == p.send_elems
        for m in p.sends:
            q = plans[m.peer]
            back = [x for x in q.recvs if x.peer == r]
            assert len(back) == 1
            assert back[0].count == m.count
            assert [s.dir for s in back[0].segments] == [s.dir for s in m.segments]
            assert [s.region.size() for s in back[0].segments] == [s.region.size() for s in m.segments]
        # Every active direction is covered exactly once (wire or self copy or PROC_NULL).
        dirs = [s.dir for m in p.sends for s in m.segments] + [c.dir for c in p.self_copies]
        assert len(dirs) == len(set(dirs))


def test_plan_2x4_peer_count_and_bytes():
    topo = C.CartTopology(2, 4)
    g = C.TileGeom.aligned(8192, 16384, 1, 1, 4)
    p = C.make_halo_plan(topo, 0, g)
    assert len(p.sends) == 5  # up == down on a 2-row torus
    # two rows of 8192 + two columns of 16384 + 4 corners
    assert p.send_elems == 2 * 8192 + 2 * 16384 + 4


def test_aligned_geometry_properties():
    for w, h, halo, eb in itertools.product([1, 7, 256, 1000], [1, 3], [1, 2], [4, 8]):
        g = C.TileGeom.aligned(w, h, halo, halo, eb)
        vec = 16 // eb
        assert (g.x_origin + g.halo_x) % vec == 0
        assert g.pitch % (256 // eb) == 0
        assert g.pitch >= g.x_origin + halo + ((w + vec - 1) // vec) * vec + vec
