// dist.cpp — transports of the partitioned MATCH exchange (dist.h).
#include "dist.h"

#include <rccl/rccl.h>

#include <cstring>
#include <string>

#include "common.h"

#define HIP_OK(x)                                                                                   \
  do {                                                                                              \
    hipError_t e_ = (x);                                                                            \
    if (e_ != hipSuccess) omx::fail(OMX_E_DEVICE, std::string(#x ": ") + hipGetErrorString(e_)); \
  } while (0)
#define NCCL_OK(x)                                                                                  \
  do {                                                                                              \
    ncclResult_t r_ = (x);                                                                          \
    if (r_ != ncclSuccess) omx::fail(OMX_E_DEVICE, std::string(#x ": ") + ncclGetErrorString(r_)); \
  } while (0)

namespace omx {

// ---- threads ----------------------------------------------------------------------------------------

ThreadHub::ThreadHub(int w) : world(w), counts(w, std::vector<uint64_t>(w, 0)), sbuf(w), sdispl(w), gathered(w) {}

void ThreadHub::barrier() {
  std::unique_lock<std::mutex> lk(m);
  if (aborted) fail(OMX_E_EXECUTION, "partitioned MATCH aborted: another rank failed");
  const uint64_t gen = generation;
  if (++arrived == world) {
    arrived = 0;
    ++generation;
    cv.notify_all();
  } else {
    cv.wait(lk, [&] { return generation != gen || aborted; });
    if (generation == gen) fail(OMX_E_EXECUTION, "partitioned MATCH aborted: another rank failed");
  }
}

void ThreadHub::abort() {
  std::lock_guard<std::mutex> lk(m);
  aborted = true;
  cv.notify_all();
}

namespace {

class ThreadTransport : public Transport {
 public:
  ThreadTransport(std::shared_ptr<ThreadHub> hub, int rank) : hub_(std::move(hub)), rank_(rank) {}
  int rank() const override { return rank_; }
  int world() const override { return hub_->world; }

  void counts(const uint64_t *d_send, std::vector<uint64_t> &send, std::vector<uint64_t> &recv,
              hipStream_t s) override {
    ++exchanges;
    const int W = world();
    send.assign(W, 0);
    HIP_OK(hipMemcpyAsync(send.data(), d_send, W * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
    {
      std::lock_guard<std::mutex> lk(hub_->m);
      hub_->counts[rank_] = send;
    }
    hub_->barrier();
    recv.assign(W, 0);
    {
      std::lock_guard<std::mutex> lk(hub_->m);
      for (int p = 0; p < W; ++p) recv[p] = hub_->counts[p][rank_];
    }
    hub_->barrier();  // the count slots may be reused
  }

  void alltoallv(const std::vector<const uint32_t *> &sbuf, const std::vector<uint64_t> &send,
                 const std::vector<uint64_t> &sdispl, const std::vector<uint32_t *> &rbuf,
                 const std::vector<uint64_t> &recv, const std::vector<uint64_t> &rdispl, hipStream_t s) override {
    (void)send;
    ++exchanges;
    const int W = world();
    HIP_OK(hipStreamSynchronize(s));  // this rank's send buffers are complete before peers read them
    {
      std::lock_guard<std::mutex> lk(hub_->m);
      hub_->sbuf[rank_] = sbuf;
      hub_->sdispl[rank_] = sdispl;
    }
    hub_->barrier();
    for (int p = 0; p < W; ++p) {
      if (!recv[p]) continue;
      const std::vector<const uint32_t *> &src = hub_->sbuf[p];
      const uint64_t off = hub_->sdispl[p][rank_];
      for (size_t c = 0; c < rbuf.size(); ++c)
        HIP_OK(hipMemcpyAsync(rbuf[c] + rdispl[p], src[c] + off, recv[p] * sizeof(uint32_t), hipMemcpyDefault, s));
    }
    HIP_OK(hipStreamSynchronize(s));
    hub_->barrier();  // peers are done reading this rank's send buffers
  }

  void abort() override { hub_->abort(); }

  std::vector<uint64_t> allgather_n(const std::vector<uint64_t> &x, hipStream_t) override {
    ++exchanges;
    {
      std::lock_guard<std::mutex> lk(hub_->m);
      hub_->gathered[rank_] = x;
    }
    hub_->barrier();
    std::vector<uint64_t> out;
    {
      std::lock_guard<std::mutex> lk(hub_->m);
      for (const auto &g : hub_->gathered) {
        if (g.size() != x.size()) fail(OMX_E_INVALID, "internal: allgather_n sizes differ between ranks");
        out.insert(out.end(), g.begin(), g.end());
      }
    }
    hub_->barrier();  // the slots may be reused
    return out;
  }

 private:
  std::shared_ptr<ThreadHub> hub_;
  int rank_;
};

// ---- RCCL -------------------------------------------------------------------------------------------

class RcclTransport : public Transport {
 public:
  RcclTransport(int rank, int world, int device, const uint8_t *id) : rank_(rank), world_(world), device_(device) {
    ncclUniqueId uid;
    static_assert(sizeof(uid.internal) == 128, "RCCL unique id size");
    std::memcpy(uid.internal, id, sizeof(uid.internal));
    HIP_OK(hipSetDevice(device));
    NCCL_OK(ncclCommInitRank(&comm_, world, uid, rank));
    HIP_OK(hipMalloc((void **)&d_recv_, std::max(1, world) * sizeof(uint64_t)));
    HIP_OK(hipMalloc((void **)&d_one_, kMaxGather * sizeof(uint64_t)));
    HIP_OK(hipMalloc((void **)&d_all_, std::max(1, world) * kMaxGather * sizeof(uint64_t)));
  }
  ~RcclTransport() override {
    (void)hipSetDevice(device_);
    if (d_recv_) (void)hipFree(d_recv_);
    if (d_one_) (void)hipFree(d_one_);
    if (d_all_) (void)hipFree(d_all_);
    if (comm_) (void)ncclCommDestroy(comm_);
  }
  // peers inside a collective with this rank are released with an error (ncclCommAbort)
  void abort() override {
    if (comm_) (void)ncclCommAbort(comm_);
    comm_ = nullptr;
  }

  std::vector<uint64_t> allgather_n(const std::vector<uint64_t> &x, hipStream_t s) override {
    ++exchanges;
    if (!comm_) fail(OMX_E_EXECUTION, "partitioned MATCH aborted: the communicator was aborted");
    const size_t n = x.size();
    if (n > kMaxGather) fail(OMX_E_INVALID, "internal: allgather_n of more than 8 words");
    if (n == 0) return {};
    HIP_OK(hipMemcpyAsync(d_one_, x.data(), n * sizeof(uint64_t), hipMemcpyHostToDevice, s));
    NCCL_OK(ncclAllGather(d_one_, d_all_, n, ncclUint64, comm_, s));
    std::vector<uint64_t> out(world_ * n);
    HIP_OK(hipMemcpyAsync(out.data(), d_all_, world_ * n * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));  // (x and out are host locals)
    return out;
  }
  int rank() const override { return rank_; }
  int world() const override { return world_; }

  void counts(const uint64_t *d_send, std::vector<uint64_t> &send, std::vector<uint64_t> &recv,
              hipStream_t s) override {
    ++exchanges;
    if (!comm_) fail(OMX_E_EXECUTION, "partitioned MATCH aborted: the communicator was aborted");
    NCCL_OK(ncclAllToAll(d_send, d_recv_, 1, ncclUint64, comm_, s));
    send.assign(world_, 0);
    recv.assign(world_, 0);
    HIP_OK(hipMemcpyAsync(send.data(), d_send, world_ * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    HIP_OK(hipMemcpyAsync(recv.data(), d_recv_, world_ * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
  }

  void alltoallv(const std::vector<const uint32_t *> &sbuf, const std::vector<uint64_t> &send,
                 const std::vector<uint64_t> &sdispl, const std::vector<uint32_t *> &rbuf,
                 const std::vector<uint64_t> &recv, const std::vector<uint64_t> &rdispl, hipStream_t s) override {
    ++exchanges;
    if (!comm_) fail(OMX_E_EXECUTION, "partitioned MATCH aborted: the communicator was aborted");
    std::vector<size_t> sc(send.begin(), send.end()), sd(sdispl.begin(), sdispl.end()), rc(recv.begin(), recv.end()),
        rd(rdispl.begin(), rdispl.end());
    NCCL_OK(ncclGroupStart());
    for (size_t c = 0; c < sbuf.size(); ++c)
      NCCL_OK(ncclAllToAllv(sbuf[c], sc.data(), sd.data(), rbuf[c], rc.data(), rd.data(), ncclUint32, comm_, s));
    NCCL_OK(ncclGroupEnd());
  }

 private:
  static constexpr size_t kMaxGather = 8;  // words per rank in one allgather_n
  int rank_, world_, device_;
  ncclComm_t comm_ = nullptr;
  uint64_t *d_recv_ = nullptr;
  uint64_t *d_one_ = nullptr, *d_all_ = nullptr;  // allgather staging
};

// ---- host collectives ------------------------------------------------------------------------------

class HostTransport : public Transport {
 public:
  HostTransport(int rank, int world, const HostCollectives &c) : rank_(rank), world_(world), c_(c) {}
  int rank() const override { return rank_; }
  int world() const override { return world_; }
  void abort() override {
    aborted_ = true;
    if (c_.abort) c_.abort(c_.ctx);
  }

  std::vector<uint64_t> allgather_n(const std::vector<uint64_t> &x, hipStream_t) override {
    ++exchanges;
    live();
    std::vector<uint64_t> out(x.size() * world_);
    if (x.empty()) return out;
    call(c_.allgather(c_.ctx, x.data(), x.size() * 8, out.data()), "allgather");
    return out;
  }

  void counts(const uint64_t *d_send, std::vector<uint64_t> &send, std::vector<uint64_t> &recv,
              hipStream_t s) override {
    ++exchanges;
    live();
    const int W = world_;
    send.assign(W, 0);
    HIP_OK(hipMemcpyAsync(send.data(), d_send, W * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
    std::vector<uint64_t> all((size_t)W * W);
    call(c_.allgather(c_.ctx, send.data(), W * 8ull, all.data()), "allgather");
    recv.assign(W, 0);
    for (int p = 0; p < W; ++p) recv[p] = all[(size_t)p * W + rank_];
  }

  // every column's rows through one host exchange: the columns' send buckets side by side per peer
  // (peer p's part = its rows of column 0, then of column 1, ...), so one callback moves them all
  void alltoallv(const std::vector<const uint32_t *> &sbuf, const std::vector<uint64_t> &send,
                 const std::vector<uint64_t> &sdispl, const std::vector<uint32_t *> &rbuf,
                 const std::vector<uint64_t> &recv, const std::vector<uint64_t> &rdispl, hipStream_t s) override {
    ++exchanges;
    live();
    const int W = world_;
    const size_t C = sbuf.size();
    uint64_t ns = 0, nr = 0;
    for (int p = 0; p < W; ++p) ns += send[p], nr += recv[p];
    std::vector<uint32_t> hs(std::max<uint64_t>(ns * C, 1)), hr(std::max<uint64_t>(nr * C, 1));
    std::vector<uint64_t> sc(W), sd(W), rc(W), rd(W);
    uint64_t o = 0;
    for (int p = 0; p < W; ++p) {
      sd[p] = o * 4;
      sc[p] = send[p] * C * 4;
      for (size_t c = 0; c < C; ++c, o += send[p])
        if (send[p]) HIP_OK(hipMemcpyAsync(hs.data() + o, sbuf[c] + sdispl[p], send[p] * 4, hipMemcpyDeviceToHost, s));
    }
    o = 0;
    for (int p = 0; p < W; ++p) {
      rd[p] = o * 4;
      rc[p] = recv[p] * C * 4;
      o += recv[p] * C;
    }
    HIP_OK(hipStreamSynchronize(s));
    call(c_.alltoallv(c_.ctx, hs.data(), sc.data(), sd.data(), hr.data(), rc.data(), rd.data()), "alltoallv");
    o = 0;
    for (int p = 0; p < W; ++p)
      for (size_t c = 0; c < C; ++c, o += recv[p])
        if (recv[p]) HIP_OK(hipMemcpyAsync(rbuf[c] + rdispl[p], hr.data() + o, recv[p] * 4, hipMemcpyHostToDevice, s));
    HIP_OK(hipStreamSynchronize(s));  // (hr is a local)
  }

 private:
  void live() const {
    if (aborted_) fail(OMX_E_EXECUTION, "partitioned MATCH aborted: the communicator was aborted");
  }
  void call(int rc, const char *what) {
    if (rc != 0) fail(OMX_E_EXECUTION, std::string("host collective ") + what + " failed (" + std::to_string(rc) + ")");
  }
  int rank_, world_;
  HostCollectives c_;
  bool aborted_ = false;
};

}  // namespace

std::unique_ptr<Transport> make_host_transport(int rank, int world, const HostCollectives &c) {
  if (world < 1 || rank < 0 || rank >= world) fail(OMX_E_INVALID, "bad communicator rank/world");
  if (!c.allgather || !c.alltoallv) fail(OMX_E_INVALID, "host collectives without allgather / alltoallv");
  return std::make_unique<HostTransport>(rank, world, c);
}

std::unique_ptr<Transport> make_thread_transport(std::shared_ptr<ThreadHub> hub, int rank) {
  return std::make_unique<ThreadTransport>(std::move(hub), rank);
}

std::unique_ptr<Transport> make_rccl_transport(int rank, int world, int device, const uint8_t *unique_id) {
  if (world < 1 || rank < 0 || rank >= world) fail(OMX_E_INVALID, "bad communicator rank/world");
  return std::make_unique<RcclTransport>(rank, world, device, unique_id);
}

void rccl_unique_id(uint8_t *out) {
  ncclUniqueId uid;
  NCCL_OK(ncclGetUniqueId(&uid));
  std::memcpy(out, uid.internal, sizeof(uid.internal));
}

}  // namespace omx
