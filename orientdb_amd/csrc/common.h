// common.h — error model and small utilities shared by the omx host runtime.
#pragma once
#include <cstdint>
#include <cstdio>
#include <stdexcept>
#include <string>
#include <vector>

#include "omx/match.h"

namespace omx {

// Every failure inside the runtime is an OmxError carrying one of the OMX_E_* codes; the C-ABI layer
// (capi.cpp) turns it into the int status + thread-local omx_last_error() message.
struct OmxError : std::runtime_error {
  int code;
  OmxError(int c, const std::string &m) : std::runtime_error(m), code(c) {}
};

[[noreturn]] inline void fail(int code, const std::string &msg) { throw OmxError(code, msg); }
[[noreturn]] inline void unsupported(const std::string &msg) { throw OmxError(OMX_E_UNSUPPORTED, msg); }

inline std::string lower(std::string s) {
  for (auto &c : s) c = (char)((c >= 'A' && c <= 'Z') ? c - 'A' + 'a' : c);
  return s;
}
inline bool ieq(const std::string &a, const std::string &b) { return lower(a) == lower(b); }

// host worker threads: the machine's CPUs, capped by OMP_NUM_THREADS (the CPU share a job gets on a
// shared box can be far below what hardware_concurrency reports) and by 64
unsigned host_threads();

inline uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

}  // namespace omx
