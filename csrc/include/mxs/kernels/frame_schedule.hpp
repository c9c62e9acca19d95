// Frame-first work schedule of the overlapped multi-GPU pass (host only, no HIP).
//
// The persistent two-stage pipeline (stencil_device.hpp) normally gives every
// workgroup an equal contiguous share of (column group x rows) in group-major
// order, so the cells a neighbour needs next — the S-deep output frame, rows
// [0, S) and [H - S, H) and columns [0, S) and [W - S, W) — are finished only
// when the pass ends, and the halo exchange of the next super-step has to wait
// for the whole pass (reference loop: exchange, then compute,
// stencil2d/mpi-2d-stencil-subarray-cuda.cu:169-172, stencil2d/stencil2D.h:363-377).
//
// This schedule hands every workgroup an explicit chunk list instead:
//   * frame chunks first: the first and last column groups (the ones holding
//     the left / right output bands) cut into short chunks of `frame_rows`
//     rows, and the top and bottom `frame_rows` rows of every other group;
//     each goes to a different workgroup as its FIRST chunk, and that
//     workgroup signals (one counter add) when it is stored;
//   * `comm_wgs` of the frame workgroups do nothing else and exit early: a
//     pipeline workgroup fills a CU (2 x 240 VGPRs per SIMD), and RCCL's
//     kernels (248-256 VGPRs per wave) only run on a CU that is free, so these
//     are the CUs the halo exchange runs on while the pass continues;
//   * the remaining rows (the middle groups' interior rows) are dealt out as
//     contiguous group-major ranges, sized so every other workgroup finishes at
//     the same time (a chunk costs its rows plus `fill` pipeline-fill rows).
// The frame is then complete after ~(frame_rows + fill) row iterations instead
// of the whole share, and pack -> RCCL send/recv -> unpack of the next halo
// runs under the rest of the pass.
#pragma once

#include <algorithm>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

namespace mxs {
namespace kernels {

struct FrameChunk {
  std::int32_t group = 0;
  std::int32_t r0 = 0, r1 = 0;  // rows [r0, r1) of the pass's row range
  std::int32_t flags = 0;       // kSignal: add 1 to the frame counter once stored
};
constexpr std::int32_t kFrameSignal = 1;

struct FrameSchedule {
  int blocks = 0;          // workgroups (table rows)
  int entries = 0;         // chunk slots per workgroup (table stride)
  int signals = 0;         // counter value once every frame chunk is stored
  int comm_wgs = 0;        // frame-only workgroups (exit early)
  std::int64_t frame_rows = 0;
  double frame_cost = 0;   // largest (frame rows + fill) of a frame chunk
  double bulk_cost = 0;    // largest total cost of a workgroup's list
  std::vector<FrameChunk> table;  // blocks x entries, unused slots r1 <= r0
  const FrameChunk& at(int wg, int e) const { return table[size_t(wg) * size_t(entries) + size_t(e)]; }
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

// groups: column groups of the pass; rows: its row count; blocks: resident
// workgroups; fill: pipeline-fill row iterations a chunk pays on top of its
// rows; frame_rows: target frame chunk height (0 = auto; at least the time
// block S, so the top / bottom frame chunks hold the S-deep bands); comm_wgs:
// frame-only workgroups; edge_left / edge_right: groups at each side that hold
// output columns of the S-wide left / right bands (2 when the last group is
// narrower than S). Throws std::invalid_argument on a degenerate request.
inline FrameSchedule make_frame_schedule(std::int64_t groups, std::int64_t rows, int blocks, std::int64_t fill,
                                         std::int64_t frame_rows = 0, int comm_wgs = 8, int edge_left = 1,
                                         int edge_right = 1) {
  if (groups <= 0 || rows <= 0 || blocks <= 0 || fill < 0)
    throw std::invalid_argument("make_frame_schedule: groups, rows and blocks must be positive");
  comm_wgs = std::max(0, comm_wgs);
  // Auto height: a frame chunk costs ~40% of an even share, so the frame is
  // stored well before the pass is half done (the exchange then has the rest
  // of the pass to run on the freed CUs), and no shorter: every frame chunk
  // pays a pipeline fill of its own.
  const double even = double(groups * rows) / blocks + double(fill);
  std::int64_t hf = frame_rows > 0 ? frame_rows : std::max<std::int64_t>(32, std::int64_t(0.4 * even) - fill);
  hf = std::min(hf, rows);
  FrameSchedule s;
  s.blocks = blocks;
  // Frame chunks. Edge groups: whole height in chunks of ~hf rows; middle
  // groups: top and bottom hf rows (the whole group when it is that short).
  // More chunks than workgroups: taller chunks until they fit.
  std::vector<FrameChunk> frame;
  std::vector<detail::Run> bulk;
  for (;;) {
    frame.clear();
    bulk.clear();
    auto cut = [&](std::int32_t g, std::int64_t r0, std::int64_t r1) {
      const std::int64_t n = std::max<std::int64_t>(1, (r1 - r0 + hf - 1) / hf);
      for (std::int64_t i = 0; i < n; ++i)
        frame.push_back(FrameChunk{g, std::int32_t(r0 + (r1 - r0) * i / n),
                                   std::int32_t(r0 + (r1 - r0) * (i + 1) / n), kFrameSignal});
    };
    for (std::int64_t g = 0; g < groups; ++g) {
      if (g < edge_left || g >= groups - edge_right || rows <= 2 * hf) {
        cut(std::int32_t(g), 0, rows);
      } else {
        frame.push_back(FrameChunk{std::int32_t(g), 0, std::int32_t(hf), kFrameSignal});
        frame.push_back(FrameChunk{std::int32_t(g), std::int32_t(rows - hf), std::int32_t(rows), kFrameSignal});
        bulk.push_back(detail::Run{std::int32_t(g), hf, rows - hf});
      }
    }
    if (std::int64_t(frame.size()) <= blocks || hf >= rows) break;
    hf = std::min(rows, hf + hf / 4 + 1);
  }
  if (std::int64_t(frame.size()) > blocks)
    throw std::invalid_argument("make_frame_schedule: " + std::to_string(frame.size()) + " frame chunks for " +
                                std::to_string(blocks) + " workgroups");
  // Frame chunk i goes to workgroup i; the first comm_wgs of them (blocks b
  // and b + 8 share an XCD: the first 8 spread over all eight) take nothing else.
  const int nf = int(frame.size());
  comm_wgs = std::min(comm_wgs, nf);
  s.comm_wgs = comm_wgs;
  s.signals = nf;
  s.frame_rows = hf;
  std::vector<std::vector<FrameChunk>> lists(static_cast<size_t>(blocks));
  std::vector<std::int64_t> load(static_cast<size_t>(blocks), 0);
  for (int i = 0; i < nf; ++i) {
    lists[size_t(i)].push_back(frame[size_t(i)]);
    load[size_t(i)] = frame[size_t(i)].r1 - frame[size_t(i)].r0 + fill;
    s.frame_cost = std::max(s.frame_cost, double(load[size_t(i)]));
  }
  // Bulk: the fill-aware greedy partition over what every workgroup has left
  // below a common finishing level T (comm workgroups: nothing).
  auto budget_t = [&](int w, std::int64_t T) -> std::int64_t {
    return w < comm_wgs ? 0 : std::max<std::int64_t>(0, T - load[size_t(w)]);
  };
  if (!bulk.empty()) {
    const std::int64_t T = detail::min_budget(bulk, blocks, fill, budget_t);
    detail::greedy_walk(bulk, blocks, fill, [&](int w) { return budget_t(w, T); },
                        [&](int w, std::int32_t g, std::int64_t r0, std::int64_t r1) {
                          lists[size_t(w)].push_back(FrameChunk{g, std::int32_t(r0), std::int32_t(r1), 0});
                          load[size_t(w)] += r1 - r0 + fill;
                        });
  }
  for (int w = 0; w < blocks; ++w) s.bulk_cost = std::max(s.bulk_cost, double(load[size_t(w)]));
  size_t entries = 1;
  for (const auto& l : lists) entries = std::max(entries, l.size());
  s.entries = int(entries);
  s.table.assign(size_t(blocks) * entries, FrameChunk{0, 0, 0, 0});
  for (int w = 0; w < blocks; ++w)
    for (size_t e = 0; e < lists[size_t(w)].size(); ++e) s.table[size_t(w) * entries + e] = lists[size_t(w)][e];
  return s;
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
  FrameSchedule inner;
  FrameSchedule outer;
  std::int64_t hf = 0;
  double inner_cost = 0, outer_cost = 0;  // slowest workgroup (rows + fills) of each set
  double serial_cost = 0;                 // the same pass as one balanced launch
};

namespace detail {
// Fill-aware partition of `runs` over `blocks` workgroups (equal budgets).
inline FrameSchedule partition_runs(const std::vector<Run>& runs, int blocks, std::int64_t fill, double* cost) {
  FrameSchedule s;
  s.blocks = blocks;
  std::vector<std::vector<FrameChunk>> lists(static_cast<size_t>(blocks));
  std::vector<std::int64_t> load(static_cast<size_t>(blocks), 0);
  if (!runs.empty()) {
    const std::int64_t T = min_budget(runs, blocks, fill, [](int, std::int64_t t) { return t; });
    greedy_walk(runs, blocks, fill, [&](int) { return T; },
                [&](int w, std::int32_t g, std::int64_t r0, std::int64_t r1) {
                  lists[size_t(w)].push_back(FrameChunk{g, std::int32_t(r0), std::int32_t(r1), 0});
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
  s.table.assign(size_t(blocks) * entries, FrameChunk{0, 0, 0, 0});
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
// lead_frac (the exchange's share of a serial pass). frame_rows: hf (0 = depth).
inline HaloLastSchedule make_halo_last_schedule(std::int64_t groups, std::int64_t rows, int blocks, std::int64_t fill,
                                                std::int64_t depth, const std::vector<std::uint8_t>& ghost_group,
                                                int outer_wgs = 0, double lead_frac = 0.12,
                                                std::int64_t frame_rows = 0, int granule = 1, int min_outer = 1) {
  if (groups <= 0 || rows <= 0 || blocks < 2 || fill < 0 || depth <= 0 || std::int64_t(ghost_group.size()) != groups)
    throw std::invalid_argument("make_halo_last_schedule: bad shape");
  HaloLastSchedule h;
  h.hf = std::max(depth, frame_rows);
  std::vector<detail::Run> inner, outer, all;
  for (std::int64_t g = 0; g < groups; ++g) {
    const auto gi = std::int32_t(g);
    all.push_back(detail::Run{gi, 0, rows});
    if (ghost_group[size_t(g)] || rows <= 2 * h.hf) {
      outer.push_back(detail::Run{gi, 0, rows});
    } else {
      outer.push_back(detail::Run{gi, 0, h.hf});
      outer.push_back(detail::Run{gi, rows - h.hf, rows});
      inner.push_back(detail::Run{gi, h.hf, rows - h.hf});
    }
  }
  if (inner.empty()) throw std::invalid_argument("make_halo_last_schedule: no interior");
  h.serial_cost = double(detail::runs_cost(all, blocks, fill));
  granule = std::max(1, granule);
  int m = outer_wgs;
  if (m <= 0) {
    // The smallest outer set whose (delayed) finish does not trail the inner set,
    // and no fewer than min_outer: the exchange's kernels run on the CUs the
    // inner launch leaves free (RCCL's p2p kernel starved on 8-16 free CUs and
    // finished only with the inner launch, profiles/r03_halolast).
    const double lead = lead_frac * h.serial_cost;
    double best = 1e300;
    const int k0 = std::max(granule, (std::max(1, min_outer) + granule - 1) / granule * granule);
    for (int k = k0; k < blocks; k += granule) {
      const double ci = double(detail::runs_cost(inner, blocks - k, fill));
      const double co = lead + double(detail::runs_cost(outer, k, fill));
      const double t = std::max(ci, co);
      if (t < best) {
        best = t;
        m = k;
      }
      if (co <= ci) break;  // more outer workgroups only slow the inner set
    }
  }
  if (m <= 0) m = std::max(granule, min_outer);
  m = std::min(std::max(m, 1), blocks - 1);
  h.inner = detail::partition_runs(inner, blocks - m, fill, &h.inner_cost);
  h.outer = detail::partition_runs(outer, m, fill, &h.outer_cost);
  return h;
}

// Both sets together cover every (group, row) exactly once; every inner chunk's
// input footprint (rows [r0 - depth, r1 + depth), a non-ghost group) is in the
// core. Returns "" or the first violation (tests).
inline std::string check_halo_last_schedule(const HaloLastSchedule& h, std::int64_t groups, std::int64_t rows,
                                            std::int64_t depth, const std::vector<std::uint8_t>& ghost_group) {
  std::vector<std::uint8_t> seen(size_t(groups * rows), 0);
  for (int set = 0; set < 2; ++set) {
    const FrameSchedule& s = set == 0 ? h.inner : h.outer;
    for (int w = 0; w < s.blocks; ++w)
      for (int e = 0; e < s.entries; ++e) {
        const FrameChunk& c = s.at(w, e);
        if (c.r1 <= c.r0) continue;
        if (c.group < 0 || c.group >= groups || c.r0 < 0 || c.r1 > rows) return "chunk out of range";
        if (c.flags != 0) return "halo-last chunks carry no signal";
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

// Every (group, row) covered exactly once, frame chunks first and signalled,
// every output frame row / edge group inside a signalled chunk. Returns "" or
// the first violation (tests).
inline std::string check_frame_schedule(const FrameSchedule& s, std::int64_t groups, std::int64_t rows,
                                        std::int64_t depth, int edge_left = 1, int edge_right = 1) {
  std::vector<std::uint8_t> seen(size_t(groups * rows), 0), framed(size_t(groups * rows), 0);
  int signals = 0;
  for (int w = 0; w < s.blocks; ++w) {
    bool bulk_started = false;
    for (int e = 0; e < s.entries; ++e) {
      const FrameChunk& c = s.at(w, e);
      if (c.r1 <= c.r0) continue;
      if (c.group < 0 || c.group >= groups || c.r0 < 0 || c.r1 > rows) return "chunk out of range";
      const bool sig = (c.flags & kFrameSignal) != 0;
      if (sig && bulk_started) return "frame chunk after a bulk chunk in workgroup " + std::to_string(w);
      if (!sig) bulk_started = true;
      signals += sig;
      for (std::int64_t r = c.r0; r < c.r1; ++r) {
        auto& v = seen[size_t(c.group * rows + r)];
        if (v) return "row covered twice";
        v = 1;
        if (sig) framed[size_t(c.group * rows + r)] = 1;
      }
    }
  }
  if (signals != s.signals) return "signal count mismatch";
  for (std::int64_t g = 0; g < groups; ++g)
    for (std::int64_t r = 0; r < rows; ++r) {
      if (!seen[size_t(g * rows + r)]) return "row not covered";
      const bool need = g < edge_left || g >= groups - edge_right || r < depth || r >= rows - depth;
      if (need && !framed[size_t(g * rows + r)]) return "frame cell outside the frame chunks";
    }
  return "";
}

}  // namespace kernels
}  // namespace mxs
