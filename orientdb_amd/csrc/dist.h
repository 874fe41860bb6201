// dist.h — the exchange step of a 1-D partitioned MATCH.
//
// The snapshot of rank r holds the out/in CSR rows of the vertices it owns; classes, RIDs and property
// columns are replicated. A binding row is expanded on the rank that owns the vertex in its source
// column, so before a step that reads the adjacency of column c, rows travel to owner(row[c]): a
// counting sort by destination rank, an all-to-all of the per-peer counts, then an all-to-all-v of
// every bound column. The reference never distributes MATCH (OMatchStatement.isLocalExecution,
// P/OMatchStatement.java:1009-1011); this is the MI355X design.
//
// Three transports implement the same two collectives:
//   * RCCL (one process per GPU, xGMI): ncclAllToAll of the counts, ncclAllToAllv of each column, on
//     the executor's stream;
//   * threads of one process (any devices, one shared GPU included): device-to-device copies between
//     the ranks' buffers behind a barrier — the single-GPU parity tests of the partitioned path run the
//     same routing code through it;
//   * processes joined by the caller's host collectives (gloo, MPI): counts and rows staged through
//     host memory — the multi-process partitioned path where the ranks' GPUs have no RCCL between them.
#pragma once
#include <hip/hip_runtime.h>

#include <condition_variable>
#include <cstdint>
#include <memory>
#include <mutex>
#include <vector>

namespace omx {

class Transport {
 public:
  virtual ~Transport() = default;
  virtual int rank() const = 0;
  virtual int world() const = 0;
  // d_send[p] (device, world words) = rows this rank sends to p; on return send/recv hold the host
  // copies of this rank's row and of what every p sends to it
  virtual void counts(const uint64_t *d_send, std::vector<uint64_t> &send, std::vector<uint64_t> &recv,
                      hipStream_t s) = 0;
  // columns: sbuf[c] holds this rank's rows bucketed by destination (send[p] rows at sdispl[p]);
  // rbuf[c] receives recv[p] rows from p at rdispl[p]. Stream-ordered on s.
  virtual void alltoallv(const std::vector<const uint32_t *> &sbuf, const std::vector<uint64_t> &send,
                         const std::vector<uint64_t> &sdispl, const std::vector<uint32_t *> &rbuf,
                         const std::vector<uint64_t> &recv, const std::vector<uint64_t> &rdispl, hipStream_t s) = 0;
  // called when this rank's execute fails: peers blocked in (or later entering) an exchange fail too
  // instead of waiting forever. The communicator is unusable afterwards.
  virtual void abort() = 0;
  // every rank's x (host values), in rank order
  std::vector<uint64_t> allgather(uint64_t x, hipStream_t s) { return allgather_n({x}, s); }
  // every rank's words x[0..n) (the same n on every rank), rank-major: out[p·n + i] = rank p's x[i] —
  // several per-level values in one host round trip
  virtual std::vector<uint64_t> allgather_n(const std::vector<uint64_t> &x, hipStream_t s) = 0;
  // collectives this rank has entered (counts / alltoallv / allgather): an execute that fails before
  // its first exchange failed the same way on every rank (the plan and its checks are replicated), so
  // nobody waits for it and the communicator stays usable
  uint64_t exchanges = 0;
};

// threads of one process as ranks
struct ThreadHub {
  explicit ThreadHub(int w);
  void barrier();  // throws OmxError once a rank has aborted
  void abort();
  const int world;
  bool aborted = false;
  std::mutex m;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t generation = 0;
  std::vector<std::vector<uint64_t>> counts;                // [src][dst]
  std::vector<std::vector<const uint32_t *>> sbuf;          // [src][column]
  std::vector<std::vector<uint64_t>> sdispl;                // [src][dst]
  std::vector<std::vector<uint64_t>> gathered;              // [src] (allgather_n)
};

std::unique_ptr<Transport> make_thread_transport(std::shared_ptr<ThreadHub> hub, int rank);
std::unique_ptr<Transport> make_rccl_transport(int rank, int world, int device, const uint8_t *unique_id);
// processes joined by the caller's host collectives (include/omx/match.h omx_host_collectives)
struct HostCollectives {
  void *ctx;
  int (*allgather)(void *, const void *, uint64_t, void *);
  int (*alltoallv)(void *, const void *, const uint64_t *, const uint64_t *, void *, const uint64_t *, const uint64_t *);
  void (*abort)(void *);
};
std::unique_ptr<Transport> make_host_transport(int rank, int world, const HostCollectives &c);
void rccl_unique_id(uint8_t *out);  // 128 bytes (NCCL_UNIQUE_ID_BYTES)

}  // namespace omx
