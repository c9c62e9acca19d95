// Chunk-list work schedules of the two-stage pipeline passes (host only, no HIP).
//
// The persistent pipeline (stencil_device.hpp) gives every workgroup a
// contiguous range of the linear (column group x rows) space. Two schedules
// are built here:
//   * balanced_starts: fill-aware equal-time shares of one whole pass (every
//     pass of the benchmarks);
//   * make_halo_last_schedule: the interior-first split of a multi-GPU
//     super-step into chunks that read only core cells and chunks that read the
//     ghost ring, run by two launches of the chunk-list kernel on disjoint CUs so
//     the halo exchange runs beside the first (reference loop: exchange, then
//     compute, stencil2d/mpi-2d-stencil-subarray-cuda.cu:169-172,
//     stencil2d/stencil2D.h:363-377).
#pragma once

#include <algorithm>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

namespace mxs {
namespace kernels {

struct PassChunk {
  std::int32_t group = 0;
  std::int32_t r0 = 0, r1 = 0;  // rows [r0, r1) of the pass's row range
  std::int32_t pad = 0;
};

struct ChunkSchedule {
  int blocks = 0;          // workgroups (table rows)
  int entries = 0;         // chunk slots per workgroup (table stride)
  double bulk_cost = 0;    // largest total cost (rows + fills) of a workgroup's list
  std::vector<PassChunk> table;  // blocks x entries, unused slots r1 <= r0
  const PassChunk& at(int wg, int e) const { return table[size_t(wg) * size_t(entries) + size_t(e)]; }
};

// Fill-aware partition of a group-major linear range of `total` rows made of
// `groups` runs of `rows` rows: consecutive workgroups take consecutive
// ranges; a range costs its rows plus `fill` per chunk (one more chunk at
// every group boundary it crosses), workgroup w has budget `budget(w, T)` and
// the partition minimises T. Equal row shares (the old rule) leave the
// workgroups whose share crosses a group boundary paying two fills: on 8192^2
// (9 groups x 8192 rows, 256 workgroups, 288-row shares, fill ~47) they need
// 382 row iterations while the rest need 335, and the pass lasts as long as
// the slowest; here every workgroup stays under ~340.
namespace detail {
struct Run {
  std::int32_t g;
  std::int64_t r0, r1;
};
// Walk the runs greedily with per-workgroup budgets; `emit(w, g, r0, r1)` for
// each chunk. Returns the rows left uncovered (0: T is feasible).
template <typename Budget, typename Emit>
std::int64_t greedy_walk(const std::vector<Run>& runs, int blocks, std::int64_t fill, Budget budget, Emit emit) {
  size_t ri = 0;
  std::int64_t pos = runs.empty() ? 0 : runs[0].r0;
  for (int w = 0; w < blocks && ri < runs.size(); ++w) {
    std::int64_t b = budget(w);
    while (b > fill && ri < runs.size()) {
      const std::int64_t take = std::min(b - fill, runs[ri].r1 - pos);
      emit(w, runs[ri].g, pos, pos + take);
      pos += take;
      b -= take + fill;
      if (pos == runs[ri].r1 && ++ri < runs.size()) pos = runs[ri].r0;
    }
  }
  std::int64_t left = 0;
  for (size_t i = ri; i < runs.size(); ++i) left += runs[i].r1 - (i == ri ? pos : runs[i].r0);
  return left;
}
// Smallest T (row iterations) for which the greedy walk covers every run.
template <typename BudgetT>
std::int64_t min_budget(const std::vector<Run>& runs, int blocks, std::int64_t fill, BudgetT budget_t) {
  std::int64_t total = 0;
  for (const auto& r : runs) total += r.r1 - r.r0;
  std::int64_t lo = 0, hi = total + 4 * fill + 1;
  auto ok = [&](std::int64_t T) {
    return greedy_walk(runs, blocks, fill, [&](int w) { return budget_t(w, T); },
                       [](int, std::int32_t, std::int64_t, std::int64_t) {}) == 0;
  };
  while (!ok(hi)) hi *= 2;
  while (lo + 1 < hi) {
    const std::int64_t mid = lo + (hi - lo) / 2;
    (ok(mid) ? hi : lo) = mid;
  }
  return hi;
}
}  // namespace detail

// Linear start index (group * rows + row) of each workgroup's range, blocks + 1
// entries (the last = groups * rows); a workgroup with nothing to do has an
// empty range.
inline std::vector<std::int64_t> balanced_starts(std::int64_t groups, std::int64_t rows, int blocks,
                                                 std::int64_t fill) {
  std::vector<detail::Run> runs;
  for (std::int64_t g = 0; g < groups; ++g) runs.push_back(detail::Run{std::int32_t(g), 0, rows});
  const std::int64_t T = detail::min_budget(runs, blocks, fill, [](int, std::int64_t t) { return t; });
  std::vector<std::int64_t> start(size_t(blocks) + 1, groups * rows);
  std::vector<std::uint8_t> seen(size_t(blocks), 0);
  detail::greedy_walk(runs, blocks, fill, [&](int) { return T; },
                      [&](int w, std::int32_t g, std::int64_t r0, std::int64_t) {
                        if (!seen[size_t(w)]) {
                          seen[size_t(w)] = 1;
                          start[size_t(w)] = std::int64_t(g) * rows + r0;
                        }
                      });
  for (int w = blocks - 1; w >= 0; --w)  // idle workgroups: empty range at the next start
    if (!seen[size_t(w)]) start[size_t(w)] = start[size_t(w) + 1];
  return start;
}

// ---------------------------------------------------------------- halo last
// Interior-first schedule of a PRE-exchange super-step (the reference's
// "exchange, then compute", stencil2d/mpi-2d-stencil-subarray-cuda.cu:169-172,
// with the compute split so the exchange hides under it). The pass is cut into
// two sets of chunks that two launches of the chunk-list kernel run on
// disjoint CUs:
//   * inner: chunks whose input footprint lies in the core (not an edge group,
//     rows [hf, rows - hf) with hf >= S): launched first, on `blocks - outer`
//     workgroups, while pack -> RCCL -> unpack of this super-step's halo runs on
//     the CUs it leaves free (a pipeline workgroup fills its CU; RCCL's kernels
//     need whole CUs);
//   * outer: the chunks that read the ghost ring (the edge groups whose joint
//     windows reach into the ghost columns, the top / bottom hf rows of the other
//     groups): launched after the unpack, on `outer` workgroups.
// `outer` is sized so that the outer set, started `lead` row iterations late
// (the exchange), ends with the inner set, in steps of `granule` workgroups:
// workgroups are dealt round-robin over the 8 XCDs, so with both launches a
// multiple of 8 every XCD holds the same split and each outer workgroup finds a
// free CU (36 outer next to 220 inner left some XCDs one CU short: that outer
// workgroup waited for an inner one and the pass took 1.7x as long).
struct HaloLastSchedule {
  ChunkSchedule inner;
  ChunkSchedule outer;
  std::int64_t hf = 0;
  double inner_cost = 0, outer_cost = 0;  // slowest workgroup (rows + fills) of each set
  double serial_cost = 0;                 // the same pass as one balanced launch
  std::int64_t band = 0;                  // rows per band of the outer set (>= hf: balance)
  std::int64_t moved_rows = 0;            // interior rows the outer launch took over (balance)
};

namespace detail {
// Fill-aware partition of `runs` over `blocks` workgroups (equal budgets).
inline ChunkSchedule partition_runs(const std::vector<Run>& runs, int blocks, std::int64_t fill, double* cost) {
  ChunkSchedule s;
  s.blocks = blocks;
  std::vector<std::vector<PassChunk>> lists(static_cast<size_t>(blocks));
  std::vector<std::int64_t> load(static_cast<size_t>(blocks), 0);
  if (!runs.empty()) {
    const std::int64_t T = min_budget(runs, blocks, fill, [](int, std::int64_t t) { return t; });
    greedy_walk(runs, blocks, fill, [&](int) { return T; },
                [&](int w, std::int32_t g, std::int64_t r0, std::int64_t r1) {
                  lists[size_t(w)].push_back(PassChunk{g, std::int32_t(r0), std::int32_t(r1), 0});
                  load[size_t(w)] += r1 - r0 + fill;
                });
  }
  double c = 0;
  size_t entries = 1;
  for (int w = 0; w < blocks; ++w) {
    c = std::max(c, double(load[size_t(w)]));
    entries = std::max(entries, lists[size_t(w)].size());
  }
  if (cost) *cost = c;
  s.entries = int(entries);
  s.bulk_cost = c;
  s.table.assign(size_t(blocks) * entries, PassChunk{0, 0, 0, 0});
  for (int w = 0; w < blocks; ++w)
    for (size_t e = 0; e < lists[size_t(w)].size(); ++e) s.table[size_t(w) * entries + e] = lists[size_t(w)][e];
  return s;
}
inline std::int64_t runs_cost(const std::vector<Run>& runs, int blocks, std::int64_t fill) {
  if (runs.empty()) return 0;
  if (blocks <= 0) return std::int64_t(1) << 40;
  return min_budget(runs, blocks, fill, [](int, std::int64_t t) { return t; });
}
}  // namespace detail

// ghost_group[g]: group g's joint windows read ghost columns (its chunks are all
// outer). depth: the time block S (hf >= depth). outer_wgs: 0 = auto from
// lead_frac (the exchange's share of a serial pass). band_rows: hf (0 = depth).
inline HaloLastSchedule make_halo_last_schedule(std::int64_t groups, std::int64_t rows, int blocks, std::int64_t fill,
                                                std::int64_t depth, const std::vector<std::uint8_t>& ghost_group,
                                                int outer_wgs = 0, double lead_frac = 0.12,
                                                std::int64_t band_rows = 0, int granule = 1, int min_outer = 1) {
  if (groups <= 0 || rows <= 0 || blocks < 2 || fill < 0 || depth <= 0 || std::int64_t(ghost_group.size()) != groups)
    throw std::invalid_argument("make_halo_last_schedule: bad shape");
  HaloLastSchedule h;
  h.hf = std::max(depth, band_rows);
  std::vector<detail::Run> inner, all;  // inner: the interior at the minimal band depth hf
  for (std::int64_t g = 0; g < groups; ++g) {
    const auto gi = std::int32_t(g);
    all.push_back(detail::Run{gi, 0, rows});
    if (!ghost_group[size_t(g)] && rows > 2 * h.hf) inner.push_back(detail::Run{gi, h.hf, rows - h.hf});
  }
  if (inner.empty()) throw std::invalid_argument("make_halo_last_schedule: no interior");
  h.serial_cost = double(detail::runs_cost(all, blocks, fill));
  granule = std::max(1, granule);
  const double lead = lead_frac * h.serial_cost;
  // The ghost-ring chunks alone are a small share of a large tile's pass (the
  // 2-GPU tile 32768 x 16384: 6%; its outer launch ended 445 us before the inner
  // one, which ran the rest on 7/8 of the CUs and lost to the serial pass,
  // profiles/r04_bal). So the outer launch takes deeper bands: rows [0, b) and
  // [rows - b, rows) of every non-edge group, b >= hf, until the two launches,
  // the outer one started `lead` late, end together. Deeper bands rather than
  // rows from elsewhere: a band chunk is one chunk either way, so its pipeline
  // fill is spread over more rows, and every inner run stays one run.
  const std::int64_t max_band = rows / 2 - 1;  // every inner run keeps >= 2 rows
  auto split = [&](std::int64_t band, std::vector<detail::Run>* in, std::vector<detail::Run>* out) {
    in->clear();
    out->clear();
    for (std::int64_t g = 0; g < groups; ++g) {
      const auto gi = std::int32_t(g);
      if (ghost_group[size_t(g)] || rows <= 2 * h.hf) {
        out->push_back(detail::Run{gi, 0, rows});
      } else {
        out->push_back(detail::Run{gi, 0, band});
        out->push_back(detail::Run{gi, rows - band, rows});
        in->push_back(detail::Run{gi, band, rows - band});
      }
    }
  };
  // Band depth for k outer workgroups: the deepest that keeps the outer
  // launch's (delayed) end at or before the inner launch's end (or one row more).
  auto balance = [&](int k, double* cost) {
    std::vector<detail::Run> in, out;
    auto times = [&](std::int64_t bd, double* ci, double* co) {
      split(bd, &in, &out);
      *ci = double(detail::runs_cost(in, blocks - k, fill));
      *co = lead + double(detail::runs_cost(out, k, fill));
    };
    double ci = 0, co = 0;
    times(h.hf, &ci, &co);
    if (co >= ci || max_band <= h.hf) {
      *cost = std::max(ci, co);
      return h.hf;
    }
    std::int64_t lo = h.hf, hi = max_band;
    while (lo < hi) {  // deepest band with co <= ci
      const std::int64_t mid = lo + (hi - lo + 1) / 2;
      times(mid, &ci, &co);
      if (co <= ci) lo = mid;
      else hi = mid - 1;
    }
    times(lo, &ci, &co);
    double best = std::max(ci, co);
    std::int64_t bd = lo;
    if (lo + 1 <= max_band) {
      double ci2 = 0, co2 = 0;
      times(lo + 1, &ci2, &co2);
      if (std::max(ci2, co2) < best) {
        best = std::max(ci2, co2);
        bd = lo + 1;
      }
    }
    *cost = best;
    return bd;
  };
  int m = outer_wgs;
  std::int64_t band = h.hf;
  if (m <= 0) {
    // The outer set with the earliest common end, no fewer than min_outer
    // workgroups: the exchange's kernels run on the CUs the inner launch leaves
    // free (RCCL's p2p kernel starved on 8-16 free CUs and finished only with
    // the inner launch, profiles/r03_halolast).
    double best = 1e300;
    const int k0 = std::max(granule, (std::max(1, min_outer) + granule - 1) / granule * granule);
    for (int k = k0; k < blocks; k += granule) {
      double t = 0;
      const std::int64_t bd = balance(k, &t);
      if (t < best - 1e-9) {
        best = t;
        m = k;
        band = bd;
      }
    }
  }
  if (m <= 0) m = std::max(granule, min_outer);
  m = std::min(std::max(m, 1), blocks - 1);
  if (outer_wgs > 0) {
    double t = 0;
    band = balance(m, &t);
  }
  std::vector<detail::Run> in, out;
  split(band, &in, &out);
  h.band = band;
  h.moved_rows = 0;
  for (const auto& r : in) h.moved_rows -= r.r1 - r.r0;
  for (const auto& r : inner) h.moved_rows += r.r1 - r.r0;
  h.inner = detail::partition_runs(in, blocks - m, fill, &h.inner_cost);
  h.outer = detail::partition_runs(out, m, fill, &h.outer_cost);
  return h;
}

// Both sets together cover every (group, row) exactly once; every inner chunk's
// input footprint (rows [r0 - depth, r1 + depth), a non-ghost group) is in the
// core. Returns "" or the first violation (tests).
inline std::string check_halo_last_schedule(const HaloLastSchedule& h, std::int64_t groups, std::int64_t rows,
                                            std::int64_t depth, const std::vector<std::uint8_t>& ghost_group) {
  std::vector<std::uint8_t> seen(size_t(groups * rows), 0);
  for (int set = 0; set < 2; ++set) {
    const ChunkSchedule& s = set == 0 ? h.inner : h.outer;
    for (int w = 0; w < s.blocks; ++w)
      for (int e = 0; e < s.entries; ++e) {
        const PassChunk& c = s.at(w, e);
        if (c.r1 <= c.r0) continue;
        if (c.group < 0 || c.group >= groups || c.r0 < 0 || c.r1 > rows) return "chunk out of range";
        if (set == 0 && (ghost_group[size_t(c.group)] || c.r0 < depth || c.r1 > rows - depth))
          return "inner chunk reads the ghost ring";
        for (std::int64_t r = c.r0; r < c.r1; ++r) {
          auto& v = seen[size_t(c.group * rows + r)];
          if (v) return "row covered twice";
          v = 1;
        }
      }
  }
  for (auto v : seen)
    if (!v) return "row not covered";
  return "";
}

}  // namespace kernels
}  // namespace mxs
