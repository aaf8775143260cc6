// MPI (host-staged) and RCCL (device-direct) communicators; see comm.hpp.
#include "comm.hpp"

#include <mpi.h>
#include <rccl/rccl.h>
#include <unistd.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>

namespace a4 {

void Comm::maybe_inject_fault(const char* what) const {
  const char* f = std::getenv("SPMM_FAULT_INJECT");
  if (!f) return;
  const std::string spec(f), want = std::string(what) + ":" + std::to_string(rank_);
  if (spec == want) throw Error("injected fault (" + spec + ")");
}

namespace {

constexpr int64_t CHUNK = int64_t(1) << 28;   // elements per MPI message (< 2^31)

#define A4_MPI(call)                                                                   \
  do {                                                                                 \
    int e_ = (call);                                                                   \
    if (e_ != MPI_SUCCESS) throw ::a4::Error(std::string("MPI error in " #call)); \
  } while (0)

template <typename T>
void mpi_send_chunks(const T* p, int64_t n, MPI_Datatype t, int dst, int tag) {
  for (int64_t o = 0; o < n; o += CHUNK)
    A4_MPI(MPI_Send(p + o, (int)std::min(CHUNK, n - o), t, dst, tag, MPI_COMM_WORLD));
}
template <typename T>
void mpi_recv_chunks(T* p, int64_t n, MPI_Datatype t, int src, int tag) {
  for (int64_t o = 0; o < n; o += CHUNK)
    A4_MPI(MPI_Recv(p + o, (int)std::min(CHUNK, n - o), t, src, tag, MPI_COMM_WORLD, MPI_STATUS_IGNORE));
}

class MpiComm : public Comm {
 public:
  MpiComm() {
    A4_MPI(MPI_Comm_rank(MPI_COMM_WORLD, &rank_));
    A4_MPI(MPI_Comm_size(MPI_COMM_WORLD, &world_));
  }
  std::string name() const override { return "mpi"; }
  void send_host(const Mat& M, int dst) override {
    maybe_inject_fault("send");
    int64_t hdr[4] = {M.rows, M.cols, M.k, M.nb()};
    A4_MPI(MPI_Send(hdr, 4, MPI_INT64_T, dst, 0, MPI_COMM_WORLD));
    mpi_send_chunks(M.keys.data(), (int64_t)M.keys.size(), MPI_INT32_T, dst, 1);
    mpi_send_chunks(M.vals.data(), (int64_t)M.vals.size(), MPI_UINT64_T, dst, 2);
    bytes_sent += M.bytes() + sizeof hdr;
  }
  Mat recv_host(int src) override {
    int64_t hdr[4];
    A4_MPI(MPI_Recv(hdr, 4, MPI_INT64_T, src, 0, MPI_COMM_WORLD, MPI_STATUS_IGNORE));
    Mat M;
    M.rows = hdr[0]; M.cols = hdr[1]; M.k = (int)hdr[2];
    M.keys.resize((size_t)hdr[3] * 2);
    M.vals.resize((size_t)hdr[3] * M.k * M.k);
    mpi_recv_chunks(M.keys.data(), (int64_t)M.keys.size(), MPI_INT32_T, src, 1);
    mpi_recv_chunks(M.vals.data(), (int64_t)M.vals.size(), MPI_UINT64_T, src, 2);
    bytes_recv += M.bytes() + sizeof hdr;
    return M;
  }
  void send_dev(const DevMat& M, int dst, hipStream_t s) override { send_host(dev_download(M, s), dst); }
  DevMat recv_dev(int src, hipStream_t s) override {
    Mat h = recv_host(src);
    DevMat d = dev_upload(h, s);
    A4_HIP(hipStreamSynchronize(s));   // h is pageable and dies here
    return d;
  }
  void barrier() override { A4_MPI(MPI_Barrier(MPI_COMM_WORLD)); }
  double allreduce_max(double x) override {
    double y = x;
    A4_MPI(MPI_Allreduce(&x, &y, 1, MPI_DOUBLE, MPI_MAX, MPI_COMM_WORLD));
    return y;
  }
  void abort(int code) override { MPI_Abort(MPI_COMM_WORLD, code); }
};

#define A4_NCCL(call)                                                                                  \
  do {                                                                                                 \
    ncclResult_t r_ = (call);                                                                          \
    if (r_ != ncclSuccess) throw ::a4::Error(std::string("RCCL error ") + ncclGetErrorString(r_) + " in " #call); \
  } while (0)

}  // namespace

void Comm::allgatherv_dev(const void* send, void* recv, const std::vector<size_t>& bytes, hipStream_t s) {
  size_t tot = 0;
  for (size_t b : bytes) tot += b;
  std::vector<char> h(std::max<size_t>(tot, 1));
  size_t at = 0;
  for (int r = 0; r < world_; ++r) {
    if (r == rank_ && bytes[r]) A4_HIP(hipMemcpyAsync(h.data() + at, send, bytes[r], hipMemcpyDeviceToHost, s));
    at += bytes[r];
  }
  A4_HIP(hipStreamSynchronize(s));
  at = 0;
  for (int r = 0; r < world_; ++r) {
    for (size_t o = 0; o < bytes[r]; o += (size_t(1) << 30)) {
      const size_t n = std::min(bytes[r] - o, size_t(1) << 30);
      A4_MPI(MPI_Bcast(h.data() + at + o, (int)n, MPI_BYTE, r, MPI_COMM_WORLD));
    }
    at += bytes[r];
  }
  if (tot) A4_HIP(hipMemcpyAsync(recv, h.data(), tot, hipMemcpyHostToDevice, s));
  A4_HIP(hipStreamSynchronize(s));
  bytes_recv += tot - bytes[rank_];
  bytes_sent += bytes[rank_];
}

namespace {

class RcclComm : public Comm {
 public:
  explicit RcclComm(double timeout_s) : timeout_s_(timeout_s) {
    A4_MPI(MPI_Comm_rank(MPI_COMM_WORLD, &rank_));
    A4_MPI(MPI_Comm_size(MPI_COMM_WORLD, &world_));
    ncclUniqueId id;
    if (rank_ == 0) A4_NCCL(ncclGetUniqueId(&id));
    A4_MPI(MPI_Bcast(&id, sizeof id, MPI_BYTE, 0, MPI_COMM_WORLD));
    A4_NCCL(ncclCommInitRank(&comm_, world_, id, rank_));
    A4_HIP(hipStreamCreateWithFlags(&own_, hipStreamNonBlocking));
    A4_HIP(hipHostMalloc(reinterpret_cast<void**>(&hhdr_), 4 * sizeof(int64_t), hipHostMallocDefault));
    A4_HIP(hipMalloc(reinterpret_cast<void**>(&dhdr_), 4 * sizeof(int64_t)));
  }
  ~RcclComm() override {
    if (comm_) ncclCommDestroy(comm_);
    if (dh_) (void)hipFree(dh_);
    if (hh_) (void)hipHostFree(hh_);
    if (dhdr_) (void)hipFree(dhdr_);
    if (hhdr_) (void)hipHostFree(hhdr_);
    if (own_) (void)hipStreamDestroy(own_);
  }
  std::string name() const override { return "rccl"; }

  void send_dev(const DevMat& M, int dst, hipStream_t s) override {
    maybe_inject_fault("send");
    arrive({dst});
    hhdr_[0] = M.rows; hhdr_[1] = M.cols; hhdr_[2] = M.k; hhdr_[3] = M.nb;
    A4_HIP(hipMemcpyAsync(dhdr_, hhdr_, 4 * sizeof(int64_t), hipMemcpyHostToDevice, s));
    A4_NCCL(ncclSend(dhdr_, 4, ncclInt64, dst, comm_, s));
    if (M.nb) {
      A4_NCCL(ncclSend(M.keys.get(), (size_t)M.nb * 2, ncclInt32, dst, comm_, s));
      A4_NCCL(ncclSend(M.vals.get(), (size_t)M.nb * M.k * M.k, ncclUint64, dst, comm_, s));
    }
    wait(s);   // the caller may free M right after
    bytes_sent += M.bytes() + 32;
  }
  DevMat recv_dev(int src, hipStream_t s) override {
    arrive({src});
    A4_NCCL(ncclRecv(dhdr_, 4, ncclInt64, src, comm_, s));
    A4_HIP(hipMemcpyAsync(hhdr_, dhdr_, 4 * sizeof(int64_t), hipMemcpyDeviceToHost, s));
    wait(s);
    DevMat M;
    M.rows = hhdr_[0]; M.cols = hhdr_[1]; M.k = (int)hhdr_[2]; M.nb = hhdr_[3];
    M.keys = DevBuf<int32_t>((size_t)M.nb * 2, s);
    M.vals = DevBuf<uint64_t>((size_t)M.nb * M.k * M.k, s);
    if (M.nb) {
      A4_NCCL(ncclRecv(M.keys.get(), (size_t)M.nb * 2, ncclInt32, src, comm_, s));
      A4_NCCL(ncclRecv(M.vals.get(), (size_t)M.nb * M.k * M.k, ncclUint64, src, comm_, s));
    }
    bytes_recv += M.bytes() + 32;
    return M;
  }
  // One group for the whole fan-out: the headers and payloads of every
  // destination are in flight together (each peer over its own xGMI link),
  // then one bounded wait.  Receivers post header then payload per source,
  // which matches the per-peer order of the grouped sends.
  void send_many_dev(const std::vector<const DevMat*>& ms, const std::vector<int>& dsts, hipStream_t s) override {
    if (ms.empty()) return;
    maybe_inject_fault("send");
    const size_t n = ms.size();
    arrive(dsts);
    ensure_hdrs(n);
    for (size_t i = 0; i < n; ++i) {
      const DevMat& M = *ms[i];
      hh_[4 * i] = M.rows; hh_[4 * i + 1] = M.cols; hh_[4 * i + 2] = M.k; hh_[4 * i + 3] = M.nb;
    }
    A4_HIP(hipMemcpyAsync(dh_, hh_, n * 4 * sizeof(int64_t), hipMemcpyHostToDevice, s));
    A4_NCCL(ncclGroupStart());
    for (size_t i = 0; i < n; ++i) {
      const DevMat& M = *ms[i];
      A4_NCCL(ncclSend(dh_ + 4 * i, 4, ncclInt64, dsts[i], comm_, s));
      if (M.nb) {
        A4_NCCL(ncclSend(M.keys.get(), (size_t)M.nb * 2, ncclInt32, dsts[i], comm_, s));
        A4_NCCL(ncclSend(M.vals.get(), (size_t)M.nb * M.k * M.k, ncclUint64, dsts[i], comm_, s));
      }
      bytes_sent += M.bytes() + 32;
    }
    A4_NCCL(ncclGroupEnd());
    wait(s);   // callers free the matrices right after
  }
  std::vector<DevMat> recv_many_dev(const std::vector<int>& srcs, hipStream_t s) override {
    const size_t n = srcs.size();
    std::vector<DevMat> out(n);
    if (!n) return out;
    arrive(srcs);
    ensure_hdrs(n);
    A4_NCCL(ncclGroupStart());
    for (size_t i = 0; i < n; ++i) A4_NCCL(ncclRecv(dh_ + 4 * i, 4, ncclInt64, srcs[i], comm_, s));
    A4_NCCL(ncclGroupEnd());
    A4_HIP(hipMemcpyAsync(hh_, dh_, n * 4 * sizeof(int64_t), hipMemcpyDeviceToHost, s));
    wait(s);
    for (size_t i = 0; i < n; ++i) {
      DevMat& M = out[i];
      M.rows = hh_[4 * i]; M.cols = hh_[4 * i + 1]; M.k = (int)hh_[4 * i + 2]; M.nb = hh_[4 * i + 3];
      M.keys = DevBuf<int32_t>((size_t)M.nb * 2, s);
      M.vals = DevBuf<uint64_t>((size_t)M.nb * M.k * M.k, s);
    }
    A4_NCCL(ncclGroupStart());
    for (size_t i = 0; i < n; ++i) {
      DevMat& M = out[i];
      if (M.nb) {
        A4_NCCL(ncclRecv(M.keys.get(), (size_t)M.nb * 2, ncclInt32, srcs[i], comm_, s));
        A4_NCCL(ncclRecv(M.vals.get(), (size_t)M.nb * M.k * M.k, ncclUint64, srcs[i], comm_, s));
      }
      bytes_recv += M.bytes() + 32;
    }
    A4_NCCL(ncclGroupEnd());
    return out;
  }
  void send_host(const Mat& M, int dst) override {
    DevMat d = dev_upload(M, own_);
    send_dev(d, dst, own_);
  }
  Mat recv_host(int src) override {
    DevMat d = recv_dev(src, own_);
    return dev_download(d, own_);
  }
  void allgatherv_dev(const void* send, void* recv, const std::vector<size_t>& bytes, hipStream_t s) override {
    maybe_inject_fault("send");
    A4_MPI(MPI_Barrier(MPI_COMM_WORLD));   // every rank has arrived: the timeout bounds the transfer only
    size_t at = 0;
    A4_NCCL(ncclGroupStart());
    for (int r = 0; r < world_; ++r) {
      if (bytes[r]) A4_NCCL(ncclBroadcast(send, (char*)recv + at, bytes[r], ncclUint8, r, comm_, s));
      at += bytes[r];
    }
    A4_NCCL(ncclGroupEnd());
    wait(s);
    bytes_recv += at - bytes[rank_];
    bytes_sent += bytes[rank_] * (world_ - 1);
  }
  void barrier() override { A4_MPI(MPI_Barrier(MPI_COMM_WORLD)); }
  double allreduce_max(double x) override {
    double y = x;
    A4_MPI(MPI_Allreduce(&x, &y, 1, MPI_DOUBLE, MPI_MAX, MPI_COMM_WORLD));
    return y;
  }
  void abort(int code) override {
    if (comm_) { ncclCommAbort(comm_); comm_ = nullptr; }
    MPI_Abort(MPI_COMM_WORLD, code);
  }

 private:
  // Arrival handshake: a zero-byte MPI token exchanged with every peer of the
  // transfer before its RCCL calls are posted.  A slow peer (skewed work,
  // rank 0 writing the output) is waited for here, without a bound, as the
  // reference's blocking MPI calls wait; a dead peer ends the job through the
  // MPI launcher.  The RCCL wait below then times only the transfer itself,
  // so a healthy but skewed job never trips the timeout.
  void arrive(const std::vector<int>& peers) {
    std::vector<MPI_Request> rq(2 * peers.size());
    char tok_out = 1;
    std::vector<char> tok_in(peers.size());
    for (size_t i = 0; i < peers.size(); ++i) {
      A4_MPI(MPI_Isend(&tok_out, 0, MPI_BYTE, peers[i], kArriveTag, MPI_COMM_WORLD, &rq[2 * i]));
      A4_MPI(MPI_Irecv(&tok_in[i], 0, MPI_BYTE, peers[i], kArriveTag, MPI_COMM_WORLD, &rq[2 * i + 1]));
    }
    if (!rq.empty()) A4_MPI(MPI_Waitall((int)rq.size(), rq.data(), MPI_STATUSES_IGNORE));
  }
  static constexpr int kArriveTag = 0x5a4;
  // Bounded wait: a peer that died leaves the stream pending forever; poll the
  // communicator's async error and give up after the timeout (fail fast).
  void wait(hipStream_t s) {
    const double t0 = now_s();
    while (true) {
      const hipError_t q = hipStreamQuery(s);
      if (q == hipSuccess) return;
      if (q != hipErrorNotReady) A4_HIP(q);
      ncclResult_t ae = ncclSuccess;
      A4_NCCL(ncclCommGetAsyncError(comm_, &ae));
      if (ae != ncclSuccess && ae != ncclInProgress)
        throw Error(std::string("RCCL async error: ") + ncclGetErrorString(ae));
      if (now_s() - t0 > timeout_s_)
        throw Error("RCCL transfer timed out after " + std::to_string(timeout_s_) + " s");
      usleep(50);
    }
  }
  // pinned host + device header slots for grouped transfers (4 int64 each)
  void ensure_hdrs(size_t n) {
    if (n <= nhdr_) return;
    if (hh_) A4_HIP(hipHostFree(hh_));
    if (dh_) A4_HIP(hipFree(dh_));
    nhdr_ = std::max<size_t>(n, 8);
    A4_HIP(hipHostMalloc(reinterpret_cast<void**>(&hh_), nhdr_ * 4 * sizeof(int64_t), hipHostMallocDefault));
    A4_HIP(hipMalloc(reinterpret_cast<void**>(&dh_), nhdr_ * 4 * sizeof(int64_t)));
  }
  size_t nhdr_ = 0;
  int64_t* hh_ = nullptr;
  int64_t* dh_ = nullptr;
  double timeout_s_;
  ncclComm_t comm_ = nullptr;
  hipStream_t own_ = nullptr;
  int64_t* hhdr_ = nullptr;
  int64_t* dhdr_ = nullptr;
};

}  // namespace

std::unique_ptr<Comm> make_mpi_comm() { return std::make_unique<MpiComm>(); }
std::unique_ptr<Comm> make_rccl_comm(double timeout_s) { return std::make_unique<RcclComm>(timeout_s); }

}  // namespace a4
