// Event-ordered caching device allocator for the native runtime (see rt.hpp).
//
// The reference allocates one 8 GB staging buffer per rank and never frees it
// (sparse_matrix_mult.cu:421-436).  The MI355X engine keeps whole chains in
// HBM and runs products of one tree level on several streams, so buffers are
// allocated on one stream (loader, producer) and released on another
// (consumer).  Ordering is explicit here:
//   release(p, s): record an event on s (the last user), cache the block;
//   alloc(n, s):   best-fit cached block; if its event has not completed, s
//                  waits on it (hipStreamWaitEvent) before any use; otherwise
//                  a fresh hipMalloc.
// Events that a stream may still be waiting on are only destroyed in trim(),
// after a device synchronise.
#include <algorithm>

#include "rt.hpp"

namespace a4 {

namespace {

size_t round_up(size_t n) {
  const size_t g = n >= (size_t(1) << 20) ? (size_t(2) << 20) : size_t(512);
  return (n + g - 1) / g * g;
}

std::vector<hipEvent_t>& retired() {
  static std::vector<hipEvent_t> r;
  return r;
}

}  // namespace

Arena& Arena::get() {
  static Arena* a = new Arena();   // never destroyed: outlives every DevBuf
  return *a;
}

void* Arena::alloc(size_t bytes, hipStream_t s) {
  const size_t need = round_up(bytes);
  std::lock_guard<std::mutex> g(mu_);
  size_t best = free_.size();
  for (size_t i = 0; i < free_.size(); ++i) {
    const size_t b = free_[i].bytes;
    if (b >= need && b <= 2 * need && (best == free_.size() || b < free_[best].bytes)) best = i;
  }
  if (best != free_.size()) {
    Block blk = free_[best];
    free_[best] = free_.back();
    free_.pop_back();
    cached_ -= blk.bytes;
    const hipError_t q = hipEventQuery(blk.ev);
    if (q == hipSuccess) {
      A4_HIP(hipEventDestroy(blk.ev));   // nobody can be waiting on it
    } else {
      if (q != hipErrorNotReady) A4_HIP(q);
      A4_HIP(hipStreamWaitEvent(s, blk.ev, 0));
      retired().push_back(blk.ev);
    }
    live_ += blk.bytes;
    peak_ = std::max(peak_, live_ + cached_);
    return blk.p;
  }
  void* p = nullptr;
  hipError_t e = hipMalloc(&p, need);
  if (e == hipErrorOutOfMemory) {   // give the cache back and retry once
    (void)hipGetLastError();
    A4_HIP(hipDeviceSynchronize());
    for (Block& b : free_) {
      A4_HIP(hipFree(b.p));
      A4_HIP(hipEventDestroy(b.ev));
    }
    free_.clear();
    cached_ = 0;
    e = hipMalloc(&p, need);
  }
  if (e != hipSuccess)
    throw Error(std::string("device allocation of ") + std::to_string(need) + " bytes failed: " +
                hipGetErrorString(e));
  live_ += need;
  peak_ = std::max(peak_, live_ + cached_);
  return p;
}

void Arena::release(void* p, size_t bytes, hipStream_t s) {
  if (!p) return;
  Block blk{p, round_up(bytes), nullptr};
  // an event creation / record failure here cannot be reported from a
  // destructor; fall back to a device-wide ordering point instead
  if (hipEventCreateWithFlags(&blk.ev, hipEventDisableTiming) != hipSuccess ||
      hipEventRecord(blk.ev, s) != hipSuccess) {
    (void)hipGetLastError();
    (void)hipDeviceSynchronize();
    if (blk.ev) (void)hipEventDestroy(blk.ev);
    (void)hipEventCreateWithFlags(&blk.ev, hipEventDisableTiming);
    (void)hipEventRecord(blk.ev, nullptr);
  }
  std::lock_guard<std::mutex> g(mu_);
  live_ -= std::min(live_, blk.bytes);
  cached_ += blk.bytes;
  free_.push_back(blk);
}

void Arena::trim() {
  A4_HIP(hipDeviceSynchronize());
  std::lock_guard<std::mutex> g(mu_);
  for (Block& b : free_) {
    A4_HIP(hipFree(b.p));
    A4_HIP(hipEventDestroy(b.ev));
  }
  free_.clear();
  cached_ = 0;
  for (hipEvent_t e : retired()) A4_HIP(hipEventDestroy(e));
  retired().clear();
}

}  // namespace a4
