// Failure detection and fault injection.
//
// The reference's policy is fail-fast: MPI_ERRORS_RETURN plus macros that
// MPI_Abort with a decoded message (mpierr.h:37-43), CUDA checks that abort
// (mpicuda3.cu:199-203), nothing for a peer that hangs. Kept here (every check
// routes to MPI_Abort under MpiEnv), plus:
//   * a communication watchdog: waits on halo messages (MPI requests, RCCL
//     streams) give up after comm_timeout() seconds with an error naming what
//     was being waited for, so a dead or stuck peer aborts the job instead of
//     hanging it (0 = wait forever, the default);
//   * a fault-injection hook, --fault-inject RANK:ITER[:exit|hang|error], to
//     check that those paths end the whole job cleanly.
#pragma once

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>

#include "mxs/core/error.hpp"

namespace mxs {

// Seconds a communication wait may take before it is treated as a failure.
inline double& comm_timeout() {
  static double t = 0.0;
  return t;
}

// Polls `done()` until it returns true; raises "<what> timed out" after
// comm_timeout() seconds (never when the timeout is 0). `on_timeout` runs
// first (e.g. ncclCommAbort) so the error path does not block on the comm.
template <typename Done, typename OnTimeout>
void wait_with_timeout(Done&& done, const char* what, OnTimeout&& on_timeout) {
  using clock = std::chrono::steady_clock;
  const double limit = comm_timeout();
  const auto t0 = clock::now();
  while (!done()) {
    const double waited = std::chrono::duration<double>(clock::now() - t0).count();
    if (limit > 0 && waited > limit) {
      on_timeout();
      raise_error(std::string(what) + " timed out after " + std::to_string(limit) +
                  " s: a peer rank is dead or hung (communication watchdog)");
    }
    // Spin for the first 20 ms (a timed window ends inside it: a 20-step
    // window on the 8-GPU tile is one ~0.3 ms pass, and a 50 us sleep -
    // 60-100 us with the scheduler - added ~20% to it; profiles/r02_window),
    // then back off so a long wait does not burn a core.
    if (waited > 0.02) std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
}

struct FaultSpec {
  enum class Kind { None, Exit, Hang, Error };
  int rank = -1;
  long long iteration = -1;
  Kind kind = Kind::None;

  bool armed() const { return kind != Kind::None; }
};

// "RANK:ITER[:exit|hang|error]" (default exit).
inline FaultSpec parse_fault_spec(const std::string& s) {
  FaultSpec f;
  if (s.empty()) return f;
  const auto c1 = s.find(':');
  MXS_CHECK(c1 != std::string::npos, "--fault-inject expects RANK:ITER[:exit|hang|error], got '" << s << "'");
  const auto c2 = s.find(':', c1 + 1);
  f.rank = std::atoi(s.substr(0, c1).c_str());
  f.iteration = std::atoll(s.substr(c1 + 1, c2 == std::string::npos ? std::string::npos : c2 - c1 - 1).c_str());
  const std::string kind = c2 == std::string::npos ? "exit" : s.substr(c2 + 1);
  if (kind == "exit") f.kind = FaultSpec::Kind::Exit;
  else if (kind == "hang") f.kind = FaultSpec::Kind::Hang;
  else if (kind == "error") f.kind = FaultSpec::Kind::Error;
  else MXS_CHECK(false, "--fault-inject: unknown fault kind '" << kind << "'");
  return f;
}

// Call once per iteration; fires on the configured rank and iteration.
inline void maybe_inject_fault(const FaultSpec& f, int rank, long long iteration) {
  if (!f.armed() || rank != f.rank || iteration != f.iteration) return;
  std::fprintf(stderr, "[fault-inject] rank %d at iteration %lld: %s\n", rank, iteration,
               f.kind == FaultSpec::Kind::Exit ? "exit" : f.kind == FaultSpec::Kind::Hang ? "hang" : "error");
  std::fflush(stderr);
  switch (f.kind) {
    case FaultSpec::Kind::Exit: std::_Exit(3);
    case FaultSpec::Kind::Hang:
      for (;;) std::this_thread::sleep_for(std::chrono::seconds(1));
    case FaultSpec::Kind::Error: raise_error("[fault-inject] injected error");
    default: break;
  }
}

}  // namespace mxs
