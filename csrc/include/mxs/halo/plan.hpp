// Halo-exchange plan (reference: TransferInfo / CreateSendRecvArrays,
// stencil2d/stencil2D.h:301-437).
//
// The reference posted one MPI message per region (8 sends + 8 receives, matched
// by tag = RegionID). RCCL has neither tags nor derived datatypes, so the plan
// here is organised per *peer*: every distinct neighbour rank gets one
// contiguous message that concatenates the segments destined to it, in the
// canonical direction order (mxs::Dir). Sender and receiver derive the same
// segment list independently:
//
//   sender r, peer p : for d in Dir order, if nbr(r, d) == p  -> send_region(d)
//   receiver p, from r: for d in Dir order, if nbr(p, -d) == r -> recv_region(-d)
//
// and nbr(r, d) == p <=> nbr(p, -d) == r on a Cartesian grid, so the lists line
// up element for element. On a 2-wide periodic dimension the "up" and "down"
// neighbours are the same rank and the message simply carries two segments;
// a neighbour that is the rank itself (periodic dimension of size 1) becomes a
// local copy. One message per peer also means one ncclSend/ncclRecv per peer,
// which is what a point-to-point xGMI mesh wants: every peer pair has its own
// link, so the messages proceed concurrently.
#pragma once

#include <algorithm>
#include <vector>

#include "mxs/grid/regions.hpp"
#include "mxs/topo/cart.hpp"

namespace mxs {

struct HaloSegment {
  int dir = 0;          // direction the data travels (sender's view)
  Array2D region;       // sender: core-edge window; receiver: ghost window
  index_t offset = 0;   // element offset inside the packed (send or recv) buffer
};

struct HaloMessage {
  int peer = kProcNull;
  index_t offset = 0;   // element offset of this message in the packed buffer
  index_t count = 0;    // elements
  std::vector<HaloSegment> segments;
};

struct HaloCopy {
  int dir = 0;   // direction from the source band to the ghost it feeds
  Array2D src;   // core-edge window
  Array2D dst;   // ghost window (opposite side)
};

struct HaloPlan {
  TileGeom tile;
  int rank = 0;
  bool corners = true;
  std::vector<HaloMessage> sends;
  std::vector<HaloMessage> recvs;
  std::vector<HaloCopy> self_copies;
  index_t send_elems = 0;
  index_t recv_elems = 0;

  int num_remote_peers() const { return int(sends.size()); }
};

// Tag of the reference's transfer for direction d: the RegionID of the core
// band it sends (stencil2d/stencil2D.h:389-391, 422, 428).
inline int reference_tag(int d) {
  static const int tags[kNumDirs] = {TOP_LEFT, TOP, TOP_RIGHT, LEFT, RIGHT, BOTTOM_LEFT, BOTTOM, BOTTOM_RIGHT};
  return tags[d];
}

// `loopback_self`: route self-neighbour data through a message to this rank
// instead of a local copy (lets a single GPU exercise the RCCL wire path with a
// 1-rank communicator, where self send/recv is legal).
inline HaloPlan make_halo_plan(const CartTopology& topo, int rank, const TileGeom& tile,
                               bool corners = true, bool loopback_self = false) {
  HaloPlan plan;
  plan.tile = tile;
  plan.rank = rank;
  plan.corners = corners;
  auto active = [&](int d) { return corners || !dir_is_corner(d); };
  if (tile.halo_x == 0 && tile.halo_y == 0) return plan;

  // Distinct remote peers in order of first appearance (deterministic on all ranks).
  std::vector<int> peers;
  for (int d = 0; d < kNumDirs; ++d) {
    if (!active(d)) continue;
    const int p = topo.neighbor(rank, d);
    if (p == kProcNull || (p == rank && !loopback_self)) continue;
    if (std::find(peers.begin(), peers.end(), p) == peers.end()) peers.push_back(p);
  }
  // Receive peers appear in the order of their opposite directions; keep the
  // same peer order for both lists so that buffer offsets are easy to reason
  // about (the set of peers is identical).
  for (int p : peers) {
    HaloMessage s;
    s.peer = p;
    s.offset = plan.send_elems;
    for (int d = 0; d < kNumDirs; ++d) {
      if (!active(d) || topo.neighbor(rank, d) != p) continue;
      HaloSegment seg{d, send_region(tile, d), s.offset + s.count};
      s.count += seg.region.size();
      s.segments.push_back(seg);
    }
    plan.send_elems += s.count;
    plan.sends.push_back(std::move(s));

    HaloMessage r;
    r.peer = p;
    r.offset = plan.recv_elems;
    for (int d = 0; d < kNumDirs; ++d) {
      if (!active(d) || topo.neighbor(rank, dir_opposite(d)) != p) continue;
      HaloSegment seg{d, recv_region(tile, dir_opposite(d)), r.offset + r.count};
      r.count += seg.region.size();
      r.segments.push_back(seg);
    }
    plan.recv_elems += r.count;
    plan.recvs.push_back(std::move(r));
  }
  for (int d = 0; d < kNumDirs && !loopback_self; ++d) {
    if (!active(d) || topo.neighbor(rank, d) != rank) continue;
    plan.self_copies.push_back(HaloCopy{d, send_region(tile, d), recv_region(tile, dir_opposite(d))});
  }
  return plan;
}

}  // namespace mxs
