// Communicators of the native `a4`.
//
// The reference ships partial products to rank 0 with blocking MPI_Send /
// MPI_Recv in three messages (header tag 0, keys tag 1 in 256 Ki chunks,
// values tag 2 in 32 MiB chunks; sparse_matrix_mult.cu:466-553).  Here a
// partial moves in the same header-then-payload protocol, but:
//   RcclComm   device-to-device over RCCL (xGMI P2P), communicator bootstrapped
//              by broadcasting the ncclUniqueId over MPI; bounded waits that
//              poll ncclCommGetAsyncError and abort on timeout
//   MpiComm    host-staged MPI (CPU engine, or GPUs shared by several ranks);
//              counts split below 2^31 elements per message (the reference's
//              int counts overflow past that, :487,504)
// Either can inject a failure for tests: SPMM_FAULT_INJECT=send:<rank> makes
// that rank fail its first send (fail-fast path, §5.3).
#pragma once

#include <memory>
#include <string>
#include <vector>

#include "rt.hpp"

namespace a4 {

class Comm {
 public:
  virtual ~Comm() = default;
  int rank() const { return rank_; }
  int world() const { return world_; }
  virtual std::string name() const = 0;
  // host matrices (CPU engine)
  virtual void send_host(const Mat& M, int dst) = 0;
  virtual Mat recv_host(int src) = 0;
  // device matrices (GPU engine), ordered on `s`
  virtual void send_dev(const DevMat& M, int dst, hipStream_t s) = 0;
  virtual DevMat recv_dev(int src, hipStream_t s) = 0;
  // fan-out / fan-in of one tree step: ms[i] to dsts[i] (any may repeat a
  // matrix), and one matrix from each of srcs.  Default: one peer at a time;
  // RCCL issues each side as ONE group (concurrent over the xGMI links) with
  // a single host wait.
  virtual void send_many_dev(const std::vector<const DevMat*>& ms, const std::vector<int>& dsts, hipStream_t s) {
    for (size_t i = 0; i < ms.size(); ++i) send_dev(*ms[i], dsts[i], s);
  }
  virtual std::vector<DevMat> recv_many_dev(const std::vector<int>& srcs, hipStream_t s) {
    std::vector<DevMat> out;
    for (int r : srcs) out.push_back(recv_dev(r, s));
    return out;
  }
  virtual void send_many_host(const std::vector<const Mat*>& ms, const std::vector<int>& dsts) {
    for (size_t i = 0; i < ms.size(); ++i) send_host(*ms[i], dsts[i]);
  }
  virtual std::vector<Mat> recv_many_host(const std::vector<int>& srcs) {
    std::vector<Mat> out;
    for (int r : srcs) out.push_back(recv_host(r));
    return out;
  }
  // all-gather of variable-size device byte buffers: rank r's `send` lands at
  // recv + (bytes[0] + .. + bytes[r - 1]).  Default: staged through host
  // memory with MPI broadcasts (1 GiB pieces, no 2^31 count limit); RCCL:
  // one grouped set of device broadcasts over xGMI and a bounded wait.
  virtual void allgatherv_dev(const void* send, void* recv, const std::vector<size_t>& bytes, hipStream_t s);
  virtual void barrier() = 0;
  virtual double allreduce_max(double x) = 0;
  virtual void abort(int code) = 0;
  size_t bytes_sent = 0, bytes_recv = 0;

 protected:
  int rank_ = 0, world_ = 1;
  void maybe_inject_fault(const char* what) const;
};

// MPI must be initialised by the caller.
std::unique_ptr<Comm> make_mpi_comm();
std::unique_ptr<Comm> make_rccl_comm(double timeout_s);

}  // namespace a4
