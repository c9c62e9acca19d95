// pingpong — GPU <-> GPU round-trip benchmark.
// Reference: test-benchmark/mpi-pingpong-gpu.cpp (blocking MPI_Send/MPI_Recv of a device
// buffer) and test-benchmark/mpi-pingpong-gpu-async.cpp (MPI_Isend/MPI_Irecv, -DHOST_COPY
// staging, -DPAGE_LOCKED pinned host buffers). The reference timed ONE round trip of ONE
// size (no warm-up); here every size gets warm-up + repetitions.
//
//   mpiexec -n 2 pingpong 1048576                       # reference: one size (doubles), PASSED/RTT
//   mpiexec -n 2 pingpong --sweep 8:268435456 --mode async --json pp.json
//   mpiexec -n 2 pingpong --transport mpi-staged --page-locked 1048576
//
// --transport rccl        ncclSend/ncclRecv between ranks 0 and 1 (xGMI); modes
//                         blocking (host-timed round trips) | async (hipEvent-timed) |
//                         overlap (async beside an ALU-bound kernel) | bidir (both ranks
//                         send at once: both directions of the link, bidir_gbps)
// --transport mpi-staged  D2H -> MPI (blocking Send/Recv, or Isend/Irecv with --mode async)
//                         -> H2D; --page-locked uses hipHostMalloc buffers (host_allocator.h)
// --transport loopback    1 rank: RCCL self send/recv; d2d / pinned / pageable: local paths
// --transport ipc         HIP IPC mailboxes: one persistent kernel per rank writes the
//                         payload straight into the peer's HBM over xGMI and spins on a
//                         system-scope flag (device-initiated, no host in the loop)
// --transport ipc-loopback 1 rank: the same kernels, ping and pong on two streams
// --transport peer-copy   the copy engines (SURVEY C16's HIP peer copy): each message is
//                         one SDMA hipMemcpyAsync into the peer's IPC-mapped mailbox, then a
//                         one-lane flag kernel; modes blocking | async | overlap | bidir
// --transport peer-copy-loopback 1 rank: the same protocol between two local mailboxes
//                         (hipMemcpyPeerAsync to the next device when there is one)
#include <mpi.h>

#include <algorithm>
#include <cstring>
#include <memory>
#include <iostream>
#include <sstream>
#include <vector>

#include "app_common.hpp"
#include "mxs/comm/mpi_env.hpp"
#include "mxs/comm/rccl_comm.hpp"
#include "mxs/core/cli.hpp"
#include "mxs/core/device.hpp"
#include "mxs/core/pinned_allocator.hpp"
#include "mxs/runtime/hip_utils.hpp"
#include "mxs/runtime/ipc.hpp"
#include "mxs/runtime/pingpong.hpp"

using namespace mxs;

namespace {

constexpr int kTag0to1 = 0x01;  // reference tags (mpi-pingpong-gpu.cpp:38-39)
constexpr int kTag1to0 = 0x10;

std::vector<size_t> parse_sweep(const std::string& s) {
  std::vector<size_t> out;
  const auto c = s.find(':');
  if (c != std::string::npos) {
    size_t lo = std::stoull(s.substr(0, c)), hi = std::stoull(s.substr(c + 1));
    for (size_t b = lo; b <= hi; b *= 2) out.push_back(b);
  } else {
    std::stringstream ss(s);
    std::string t;
    while (std::getline(ss, t, ',')) out.push_back(std::stoull(t));
  }
  return out;
}

// Host-staged round trip (HOST_COPY): the reference's async variant.
template <typename HostVec>
PingPongStats staged(const MpiEnv& env, HostVec& hsend, HostVec& hrecv, void* dsend, void* drecv, size_t bytes,
                     int warmup, int reps, bool async) {
  PingPongStats st;
  st.bytes = bytes;
  const int me = env.rank(), peer = 1 - me;
  std::vector<unsigned char> pattern(bytes);
  for (size_t i = 0; i < bytes; ++i) pattern[i] = static_cast<unsigned char>((i * 131u + 7u) % 251u);
  if (me == 0) MXS_HIP_CHECK(hipMemcpy(dsend, pattern.data(), bytes, hipMemcpyHostToDevice));
  auto xfer = [&](void* buf, bool send, int tag) {
    if (!async) {
      if (send) MXS_MPI_CHECK(MPI_Send(buf, int(bytes), MPI_BYTE, peer, tag, MPI_COMM_WORLD));
      else MXS_MPI_CHECK(MPI_Recv(buf, int(bytes), MPI_BYTE, peer, tag, MPI_COMM_WORLD, MPI_STATUS_IGNORE));
    } else {
      MPI_Request r;
      if (send) MXS_MPI_CHECK(MPI_Isend(buf, int(bytes), MPI_BYTE, peer, tag, MPI_COMM_WORLD, &r));
      else MXS_MPI_CHECK(MPI_Irecv(buf, int(bytes), MPI_BYTE, peer, tag, MPI_COMM_WORLD, &r));
      MXS_MPI_CHECK(MPI_Wait(&r, MPI_STATUS_IGNORE));
    }
  };
  std::vector<double> rtt;
  for (int i = 0; i < warmup + reps; ++i) {
    const double t0 = MPI_Wtime();
    if (me == 0) {
      MXS_HIP_CHECK(hipMemcpy(hsend.data(), dsend, bytes, hipMemcpyDeviceToHost));
      xfer(hsend.data(), true, kTag0to1);
      xfer(hrecv.data(), false, kTag1to0);
      MXS_HIP_CHECK(hipMemcpy(drecv, hrecv.data(), bytes, hipMemcpyHostToDevice));
    } else {
      xfer(hrecv.data(), false, kTag0to1);
      MXS_HIP_CHECK(hipMemcpy(drecv, hrecv.data(), bytes, hipMemcpyHostToDevice));
      MXS_HIP_CHECK(hipMemcpy(hsend.data(), drecv, bytes, hipMemcpyDeviceToHost));
      xfer(hsend.data(), true, kTag1to0);
    }
    if (i >= warmup) rtt.push_back((MPI_Wtime() - t0) * 1e6);
  }
  std::sort(rtt.begin(), rtt.end());
  st.reps = int(rtt.size());
  st.min_rtt_us = rtt.front();
  st.max_rtt_us = rtt.back();
  st.median_rtt_us = rtt[rtt.size() / 2];
  if (me == 0) {
    std::vector<unsigned char> back(bytes);
    MXS_HIP_CHECK(hipMemcpy(back.data(), drecv, bytes, hipMemcpyDeviceToHost));
    st.verified = std::equal(back.begin(), back.end(), pattern.begin());
  } else {
    st.verified = true;
  }
  return st;
}

}  // namespace

int main(int argc, char** argv) {
  MpiEnv env(&argc, &argv);
  Cli cli(argc, argv, {"page-locked", "host-copy", "quiet"});
  const DeviceBinding dev = bind_device(env, cli.get("bind", "bunch"));
  const auto& pos = cli.positional();
  std::vector<size_t> sizes;
  if (!pos.empty()) sizes.push_back(size_t(std::stoull(pos[0])) * sizeof(double));
  else sizes = parse_sweep(cli.get("sweep", "8:268435456"));
  std::string transport = cli.get("transport", "auto");
  if (cli.flag("host-copy")) transport = "mpi-staged";
  if (transport == "auto") transport = env.size() >= 2 ? (dev.shared ? "mpi-staged" : "rccl")
                                                         : "loopback";
  const std::string mode = cli.get("mode", "blocking");
  const int warmup = int(cli.get_int("warmup", 5)), reps = int(cli.get_int("reps", 20));
  if (env.size() < 2 &&
      (transport == "rccl" || transport == "mpi-staged" || transport == "ipc" || transport == "peer-copy")) {
    if (env.rank() == 0) std::cerr << "transport " << transport << " needs 2 ranks" << std::endl;
    return 1;
  }
  const size_t maxb = *std::max_element(sizes.begin(), sizes.end());
  DeviceBuffer<unsigned char> dsend(static_cast<index_t>(maxb)), drecv(static_cast<index_t>(maxb));
  Stream stream;
  std::unique_ptr<RcclComm> comm;
  if (transport == "rccl" || transport == "loopback") {
    std::string uid = env.rank() == 0 ? RcclComm::make_unique_id() : std::string(sizeof(ncclUniqueId), '\0');
    MXS_MPI_CHECK(MPI_Bcast(&uid[0], int(uid.size()), MPI_BYTE, 0, MPI_COMM_WORLD));
    comm = std::make_unique<RcclComm>(uid, env.size(), env.rank());
  }
  std::vector<unsigned char, PinnedAllocator<unsigned char>> pin_s, pin_r;
  std::vector<unsigned char> pg_s, pg_r;
  const bool pinned = cli.flag("page-locked");
  if (transport == "mpi-staged") {
    if (pinned) {
      pin_s.resize(maxb);
      pin_r.resize(maxb);
    } else {
      pg_s.resize(maxb);
      pg_r.resize(maxb);
    }
  }
  const bool active = env.rank() < 2;
  // HIP IPC: mailboxes exchanged between ranks 0 and 1 (runtime/ipc.hpp).
  std::unique_ptr<IpcMailbox> mailbox;
  std::unique_ptr<IpcPeerMailbox> peer_box;
  if ((transport == "ipc" || transport == "peer-copy") && active) {
    mailbox = std::make_unique<IpcMailbox>(maxb);
    std::string mine = mailbox->handle(), theirs(mine.size(), '\0');
    const int other = 1 - env.rank();
    MXS_MPI_CHECK(MPI_Sendrecv(&mine[0], int(mine.size()), MPI_BYTE, other, 7, &theirs[0], int(theirs.size()),
                               MPI_BYTE, other, 7, MPI_COMM_WORLD, MPI_STATUS_IGNORE));
    peer_box = std::make_unique<IpcPeerMailbox>(theirs);
    std::vector<unsigned char> pattern(maxb);
    for (size_t i = 0; i < maxb; ++i) pattern[i] = static_cast<unsigned char>((i * 131 + 7) % 251);
    MXS_HIP_CHECK(hipMemcpy(dsend.get(), pattern.data(), maxb, hipMemcpyHostToDevice));
  }
  const PingPongMode m = mode == "async"     ? PingPongMode::Async
                       : mode == "overlap" ? PingPongMode::Overlap
                       : mode == "bidir"   ? PingPongMode::Bidirectional
                                           : PingPongMode::Blocking;
  for (size_t bytes : sizes) {
    PingPongStats st;
    if (!active) continue;
    if (transport == "rccl" || transport == "loopback") {
      const int peer = transport == "loopback" ? env.rank() : 1 - env.rank();
      st = pingpong_rccl(*comm, peer, dsend.get(), drecv.get(), bytes, warmup, reps, m, stream.get());
    } else if (transport == "ipc") {
      IpcPingPongConfig c;
      c.bytes = bytes;
      c.warmup = warmup;
      c.reps = std::max(reps, 1);
      char token = 0;
      const int other = 1 - env.rank();
      MXS_MPI_CHECK(MPI_Sendrecv(&token, 1, MPI_BYTE, other, 8, &token, 1, MPI_BYTE, other, 8, MPI_COMM_WORLD,
                                 MPI_STATUS_IGNORE));
      st = pingpong_ipc(*mailbox, peer_box->base(), dsend.get(), env.rank() == 0, c, stream.get());
      MXS_HIP_CHECK(hipMemcpy(drecv.get(), mailbox->data(), bytes, hipMemcpyDeviceToDevice));
    } else if (transport == "ipc-loopback") {
      st = pingpong_ipc_loopback(bytes, warmup, std::max(reps, 1));
    } else if (transport == "peer-copy") {
      PeerCopyConfig c;
      c.bytes = bytes;
      c.warmup = warmup;
      c.reps = std::max(reps, 1);
      c.mode = m;
      st = pingpong_peer_copy(*mailbox, peer_box->base(), dsend.get(), env.rank() == 0, c, stream.get());
      MXS_HIP_CHECK(hipMemcpy(drecv.get(), mailbox->data(), bytes, hipMemcpyDeviceToDevice));
    } else if (transport == "peer-copy-loopback") {
      int n = 1;
      MXS_HIP_CHECK(hipGetDeviceCount(&n));
      st = pingpong_peer_copy_local(bytes, warmup, std::max(reps, 1), dev.device, (dev.device + 1) % std::max(n, 1));
    } else if (transport == "mpi-staged") {
      st = pinned ? staged(env, pin_s, pin_r, dsend.get(), drecv.get(), bytes, warmup, reps, mode == "async")
                  : staged(env, pg_s, pg_r, dsend.get(), drecv.get(), bytes, warmup, reps, mode == "async");
    } else {
      const LocalPath p = transport == "d2d" ? LocalPath::DeviceCopy
                        : transport == "pinned" ? LocalPath::PinnedStaging : LocalPath::PageableStaging;
      st = pingpong_local(p, dsend.get(), drecv.get(), bytes, warmup, reps, stream.get());
    }
    if (env.rank() != 0) continue;
    if (!pos.empty()) {
      // Reference output block (mpi-pingpong-gpu.cpp:58-71).
      if (!st.verified) {
        std::cout << "FAILED" << std::endl;
        continue;
      }
      std::cout << "PASSED\n";
      if (bytes < 1024 * 1024) std::cout << "Message size(bytes): " << bytes << '\n';
      else std::cout << "Message size(MB): " << (bytes / (1024 * 1024.0)) << '\n';
      std::cout << "Round-trip time(ms): " << st.median_rtt_us / 1000.0 << '\n';
      // D2H of the received buffer, timed like the reference's second interval.
      std::vector<unsigned char> h(bytes);
      const double t0 = MPI_Wtime();
      MXS_HIP_CHECK(hipMemcpy(h.data(), drecv.get(), bytes, hipMemcpyDeviceToHost));
      std::cout << "Device to host transfer time(ms): " << (MPI_Wtime() - t0) * 1000.0 << std::endl;
    }
    std::ostringstream js;
    js << "{\"app\": \"pingpong\", \"transport\": \"" << transport << "\", \"mode\": \"" << mode
       << "\", \"bytes\": " << bytes << ", \"rtt_us\": " << app::fmt(st.median_rtt_us)
       << ", \"rtt_min_us\": " << app::fmt(st.min_rtt_us) << ", \"latency_us\": " << app::fmt(st.latency_us())
       << ", \"gbps\": " << app::fmt(st.bandwidth_gbps()) << ", \"reps\": " << st.reps
       << ", \"passed\": " << (st.verified ? "true" : "false");
    js << ", \"timing\": \"" << (mode == "blocking" ? "host" : "device") << "\"";
    if (mode == "bidir") js << ", \"bidir_gbps\": " << app::fmt(st.bidir_gbps());
    if (mode == "overlap")
      js << ", \"compute_alone_us\": " << app::fmt(st.compute_alone_us) << ", \"comm_alone_us\": "
         << app::fmt(st.comm_alone_us) << ", \"overlapped_us\": " << app::fmt(st.overlapped_us);
    js << app::meta_json(device_description(dev.device)) << "}";
    if (pos.empty() && !cli.flag("quiet")) std::cout << js.str() << std::endl;
    app::append_json(cli.get("json"), js.str());
  }
  comm.reset();
  return 0;
}
